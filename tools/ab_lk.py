"""A/B timing of C2 lookupN(3) variants in ONE process, interleaved rounds (round 5).

    python tools/ab_lk.py --variants '{"base": {}, "al": {"RP_LOOKUP_AL": "1"}}' [--rounds 7] [--log2 26]

Each variant is a set of environment knobs read by the launcher at call time. The C2 ring
(10k servers x 100 points) and 2^26 device keys are built once. Every variant's output digest is
printed next to the base variant's (diagnostic ablations, RP_LOOKUP_ABLATE, are expected to
differ). Times: HIP events around the whole op (kernel + deferred pass), median / min over rounds.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

KNOBS = ("RP_LOOKUP_HALF", "RP_LOOKUP_LEAN", "RP_LOOKUP_KPL", "RP_RING_LAYOUT", "RP_LOOKUP_ABLATE", "RP_RING_WIDE",
         "RP_LOOKUP_GRID", "RP_LOOKUP_STG", "RP_LOOKUP_LH", "RP_LOOKUP_STGHS", "RP_LOOKUP_WPRED",
         "RP_LOOKUP_FUSEFIX", "RP_LOOKUP_HINT", "RP_LOOKUP_AL")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", required=True)
    ap.add_argument("--servers", type=int, default=10000)
    ap.add_argument("--log2", type=int, default=26)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    variants = json.loads(a.variants)
    rpa = bench.load_pkg()
    ring = rpa.HashRing()
    ring.addRemoveServers([bench.c2_addr(i) for i in range(a.servers)])
    B = 1 << a.log2
    st = torch.cuda.current_stream()
    keys = torch.empty(B * 36, dtype=torch.uint8, device="cuda")
    rpa.gen_uuid_keys_dev(42, 0, B, keys.data_ptr(), st.cuda_stream)
    out = torch.empty(B * 3, dtype=torch.int32, device="cuda")
    w = torch.arange(B * 3, device="cuda") % 1009 + 1
    times = {k: [] for k in variants}
    digests = {}
    for r in range(a.rounds + 1):
        for name, env in variants.items():
            for kn in KNOBS:
                os.environ.pop(kn, None)
            os.environ.update(env)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            ring.lookupn_dev(keys.data_ptr(), B, 3, out.data_ptr(), None, 36, None, st.cuda_stream)
            e1.record(st)
            torch.cuda.synchronize()
            if r:
                times[name].append(e0.elapsed_time(e1))
            else:
                digests[name] = int(torch.sum(out.long() * w).item())
        print("round %d done" % r, flush=True)
    for kn in KNOBS:
        os.environ.pop(kn, None)
    res = {}
    first = next(iter(variants))
    for name, t in times.items():
        med = float(np.median(t))
        res[name] = {"env": variants[name], "median_ms": round(med, 4), "min_ms": round(float(np.min(t)), 4),
                     "G_lookupN3_s": round(B / med / 1e6, 2), "hbm_frac": round(48 * B / (med * 1e-3) / 1e9 / 8000, 4),
                     "same_as_" + first: digests[name] == digests[first]}
    txt = json.dumps(res, indent=1)
    print(txt)
    if a.out:
        os.makedirs(os.path.dirname(a.out), exist_ok=True)
        with open(a.out, "w") as f:
            f.write(txt + "\n")


if __name__ == "__main__":
    main()
