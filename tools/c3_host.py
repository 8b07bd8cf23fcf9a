"""C3 host enqueue rate: with the GPU held by a spin kernel, how long the host takes to enqueue N
checksummed update batches (update_dev), per batch, for the string writer on the build stream
(RP_MEMBERS_SIDE_BUILD=1) and on the caller's stream (0); then the GPU time of the same batches
once released. If the host's per-batch time is at or above the GPU's, the stream is host-bound.

    python tools/c3_host.py [--batches 256]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=256)
    ap.add_argument("--rounds", type=int, default=2)
    a = ap.parse_args()
    import torch
    rpa = bench.load_pkg()
    S = bench._synth()
    n = k = 100_000
    names, st0, inc0 = S.c3_members(n)
    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream
    sets = []
    for q in range(16):
        ids, us, ui = S.c3_updates(n, k, seed=100 + q, base_inc=inc0 + 3 * q)
        sets.append((torch.from_numpy(ids.view(np.int32)).cuda(), torch.from_numpy(us).cuda(), torch.from_numpy(ui).cuda()))
    app = torch.empty(k, dtype=torch.uint8, device="cuda")
    na = torch.zeros(1, dtype=torch.int32, device="cuda")
    res = {}
    for r in range(a.rounds):
        for side in ("1", "0"):
            os.environ["RP_MEMBERS_SIDE_BUILD"] = side
            m = rpa.Membership(whoami=names[0], capacity=n)
            ids0 = np.asarray(m.intern(names), dtype=np.uint32)
            m.update_ids(ids0, st0, inc0, now_ms=1)
            lap = [0]

            def one(b):
                d = sets[b % len(sets)]
                inc = d[2] + 3 * len(sets) * (b // len(sets) + lap[0])
                m.update_dev(d[0].data_ptr(), d[1].data_ptr(), inc.data_ptr(), k, 1434500000000 + b, app.data_ptr(),
                             None, None, na.data_ptr(), sp)
            for b in range(8):
                one(b)
            _ = m.checksum
            torch.cuda.synchronize()
            incs = None  # (the incarnation tensors above are made per call: keep that cost out)
            pre = [(d[0], d[1], d[2] + 3 * len(sets) * (1 + b // len(sets))) for b, d in
                   enumerate([sets[b % len(sets)] for b in range(a.batches)])]

            def one2(b):
                d = pre[b]
                m.update_dev(d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), k, 1434500000100 + b, app.data_ptr(),
                             None, None, na.data_ptr(), sp)
            torch.cuda._sleep(200_000_000)  # hold the GPU while the host enqueues
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            t0 = time.perf_counter()
            for b in range(a.batches):
                one2(b)
            host_us = (time.perf_counter() - t0) * 1e6 / a.batches
            ck = m.checksum
            e1.record(stream)
            torch.cuda.synchronize()
            res.setdefault(side, []).append({"host_us_per_batch": host_us, "checksum": ck})
            print("side", side, r, json.dumps(res[side][-1]), flush=True)
            m.close()
            del pre, incs
    print(json.dumps(res))


if __name__ == "__main__":
    main()
