"""A/B of the compact layout's bucket density (RP_COMPACT_CB_DELTA at ring build) and keys per
lane, interleaved rounds in one process. python tools/ab_cb.py [--servers 10000]"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--servers", type=int, default=10000)
ap.add_argument("--rounds", type=int, default=7)
a = ap.parse_args()
rpa = bench.load_pkg()
servers = [bench.c2_addr(i) for i in range(a.servers)]
rings = {}
for d in os.environ.get("AB_CB_DELTAS", "0").split(","):
    os.environ["RP_COMPACT_CB_DELTA"] = d
    r = rpa.HashRing()
    r.addRemoveServers(servers)
    rings[d] = r
os.environ.pop("RP_COMPACT_CB_DELTA")
B = 1 << 26
st = torch.cuda.current_stream()
keys = torch.empty(B * 36, dtype=torch.uint8, device="cuda")
rpa.gen_uuid_keys_dev(42, 0, B, keys.data_ptr(), st.cuda_stream)
out = torch.empty(B * 3, dtype=torch.int32, device="cuda")
ref = None
times = {}
for rd in range(a.rounds + 1):
    for d, r in rings.items():
        for kpl in os.environ.get("AB_CB_KPL", "4,2").split(","):
            os.environ["RP_LOOKUP_KPL"] = kpl[0]
            os.environ["RP_LOOKUP_ABLATE"] = kpl[2:] if "a" in kpl else "0"
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            r.lookupn_dev(keys.data_ptr(), B, 3, out.data_ptr(), None, 36, None, st.cuda_stream)
            e1.record(st)
            torch.cuda.synchronize()
            if rd:
                times.setdefault("cb%+d/kpl%s" % (int(d), kpl), []).append(e0.elapsed_time(e1))
            if rd == 1 and "a" not in kpl:
                h = int(torch.sum(out[: 1 << 22].to(torch.int64) * 2654435761 % 1000003).item())
                ref = h if ref is None else ref
                assert h == ref, "results differ between layouts"
for k, t in times.items():
    med = float(np.median(t))
    print("%-14s %.3f ms %6.0f GB/s" % (k, med, 48 * B / med / 1e6))
