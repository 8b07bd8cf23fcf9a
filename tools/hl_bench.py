"""Chain kernels alone: rp_hash32_long_multi_dev on n strings of L bytes (the C3 checksum groups:
128 strings of ~3.6 MB), packed (k_hash_long_pack, 16 a workgroup) against one workgroup a
string, HIP events, alternating.

    python tools/hl_bench.py [--len 3600000] [--n 128,256,512] [--reps 3]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--len", type=int, default=3_600_000)
    ap.add_argument("--n", default="128,256,512")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import numpy as np
    import torch
    rpa = bench.load_pkg()
    stride = ((a.len + 32 + 255) // 256) * 256
    nmax = max(int(x) for x in a.n.split(","))
    buf = torch.randint(32, 127, (stride * nmax,), dtype=torch.uint8, device="cuda")
    res = {}
    for r in range(a.reps):
        for n in (int(x) for x in a.n.split(",")):
            for pack in ("1", "0"):
                os.environ["RP_HL_PACK"] = pack
                meta = np.zeros(4 * n, dtype=np.uint32)
                meta[0::4] = a.len + 1
                meta[1::4] = 1
                d_m = torch.from_numpy(meta.view(np.int32)).cuda()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                rpa.check(rpa.lib().rp_hash32_long_multi_dev(buf.data_ptr(), stride, n, d_m.data_ptr(), None))
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1)
                h = d_m.cpu().numpy().view(np.uint32)[2::4]
                key = "n%d/%s" % (n, "pack" if pack == "1" else "wg")
                res.setdefault(key, []).append(ms)
                res.setdefault(key + "/digest", int(h.astype(np.uint64).sum()))
                print(key, round(ms, 3), "ms", flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
