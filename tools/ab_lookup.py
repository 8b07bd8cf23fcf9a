"""A/B timing of lookupN kernels in ONE process, interleaved rounds (guide §5.4 rule 24).

    python tools/ab_lookup.py [--servers 10000] [--log2 26] [--rounds 7]

Variants: the compact layout through the lean kernel (default) and the round-1 kernel
(RP_LOOKUP_LEAN=0) at 1/2/3/4/8 keys per lane, the packed probe kernel
(RP_RING_LAYOUT=packed), the wide binary-search kernel (RP_RING_WIDE=1), and the hash-only
ablation, for lookup and lookupN(3). Prints median/min ms and lookups/s per variant.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--servers", type=int, default=10000)
    ap.add_argument("--log2", type=int, default=26)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--only", default="", help="comma-separated variant names")
    a = ap.parse_args()
    rpa = bench.load_pkg()
    ring = rpa.HashRing()
    ring.addRemoveServers([bench.c2_addr(i) for i in range(a.servers)])
    B = 1 << a.log2
    st = torch.cuda.current_stream()
    keys = torch.empty(B * 36, dtype=torch.uint8, device="cuda")
    rpa.gen_uuid_keys_dev(42, 0, B, keys.data_ptr(), st.cuda_stream)
    out = torch.empty(B * 3, dtype=torch.int32, device="cuda")
    # name -> (environment, n): compact = the default layout; packed = RP_RING_LAYOUT=packed
    variants = {
        "compact-kpl4/lookupN3": ({"RP_LOOKUP_LEAN": "0", "RP_LOOKUP_KPL": "4"}, 3),
        "compact-kpl2/lookupN3": ({"RP_LOOKUP_LEAN": "0", "RP_LOOKUP_KPL": "2"}, 3),
        "compact-kpl1/lookupN3": ({"RP_LOOKUP_LEAN": "0", "RP_LOOKUP_KPL": "1"}, 3),
        "lean-kpl4/lookupN3": ({"RP_LOOKUP_HALF": "0", "RP_LOOKUP_KPL": "4"}, 3),
        "default/lookupN3": ({}, 3),
        "stg1/lookupN3": ({"RP_LOOKUP_STG": "1"}, 3),
        "lh2/lookupN3": ({"RP_LOOKUP_LH": "2"}, 3),
        "stg2/lookupN3": ({"RP_LOOKUP_STG": "2"}, 3),
        "stg2-lh1/lookupN3": ({"RP_LOOKUP_STG": "2", "RP_LOOKUP_LH": "1"}, 3),
        "stg2-hs4/lookupN3": ({"RP_LOOKUP_STG": "2", "RP_LOOKUP_STGHS": "4"}, 3),
        "lean-kpl2/lookupN3": ({"RP_LOOKUP_LEAN": "1", "RP_LOOKUP_KPL": "2"}, 3),
        "half-kpl4/lookupN3": ({"RP_LOOKUP_HALF": "2", "RP_LOOKUP_KPL": "4"}, 3),
        "half-kpl8/lookupN3": ({"RP_LOOKUP_HALF": "2", "RP_LOOKUP_KPL": "8"}, 3),
        "quarter-kpl8/lookupN3": ({"RP_LOOKUP_HALF": "4", "RP_LOOKUP_KPL": "8"}, 3),
        "quarter-kpl4/lookupN3": ({"RP_LOOKUP_HALF": "4", "RP_LOOKUP_KPL": "4"}, 3),
        "half-kpl2/lookupN3": ({"RP_LOOKUP_HALF": "2", "RP_LOOKUP_KPL": "2"}, 3),
        "lean-kpl3/lookupN3": ({"RP_LOOKUP_LEAN": "1", "RP_LOOKUP_KPL": "3"}, 3),
        "compact-kpl3/lookupN3": ({"RP_LOOKUP_LEAN": "0", "RP_LOOKUP_KPL": "3"}, 3),
        "lean-kpl8/lookupN3": ({"RP_LOOKUP_HALF": "1", "RP_LOOKUP_KPL": "8"}, 3),
        "compact-kpl4/lookup": ({"RP_LOOKUP_LEAN": "0", "RP_LOOKUP_KPL": "4"}, 1),
        "lean-kpl4/lookup": ({"RP_LOOKUP_LEAN": "1", "RP_LOOKUP_KPL": "4"}, 1),
        "compact-kpl2/lookup": ({"RP_LOOKUP_LEAN": "0", "RP_LOOKUP_KPL": "2"}, 1),
        "probe/lookupN3": ({"RP_RING_LAYOUT": "packed", "RP_LOOKUP_KPL": "2"}, 3),
        "probe/ablate-hash-only": ({"RP_RING_LAYOUT": "packed", "RP_LOOKUP_ABLATE": "1"}, 3),
        "wide/lookupN3": ({"RP_RING_WIDE": "1"}, 3),
        "grid1024/lookupN3": ({"RP_LOOKUP_GRID": "1024"}, 3),
        "grid4096/lookupN3": ({"RP_LOOKUP_GRID": "4096"}, 3),
        "grid8192/lookupN3": ({"RP_LOOKUP_GRID": "8192"}, 3),
        "grid3072/lookupN3": ({"RP_LOOKUP_GRID": "3072"}, 3),
        "grid5120/lookupN3": ({"RP_LOOKUP_GRID": "5120"}, 3),
        "grid6144/lookupN3": ({"RP_LOOKUP_GRID": "6144"}, 3),
        "grid16384/lookupN3": ({"RP_LOOKUP_GRID": "16384"}, 3),
        "grid32768/lookupN3": ({"RP_LOOKUP_GRID": "32768"}, 3),
        # round 6: the LDS-index kernel against the lean kernel
        "lds/lookupN3": ({"RP_LOOKUP_LDS": "1"}, 3),
        "lean/lookupN3": ({"RP_LOOKUP_LDS": "0"}, 3),
        "lds/lookup": ({"RP_LOOKUP_LDS": "1"}, 1),
        "lean/lookup": ({"RP_LOOKUP_LDS": "0"}, 1),
        "lds-g512/lookupN3": ({"RP_LOOKUP_LDS": "1", "RP_LOOKUP_LDS_GRID": "512"}, 3),
        "lds-g128/lookupN3": ({"RP_LOOKUP_LDS": "1", "RP_LOOKUP_LDS_GRID": "128"}, 3),
        "lds-stg1/lookupN3": ({"RP_LOOKUP_LDS": "1", "RP_LOOKUP_LDS_STG": "1"}, 3),
        "lds-abl1/lookupN3": ({"RP_LOOKUP_LDS": "1", "RP_LOOKUP_LDS_ABL": "1"}, 3),
        "lds-abl2/lookupN3": ({"RP_LOOKUP_LDS": "1", "RP_LOOKUP_LDS_ABL": "2"}, 3),
        "lds-abl3/lookupN3": ({"RP_LOOKUP_LDS": "1", "RP_LOOKUP_LDS_ABL": "3"}, 3),
        "lds-abl4/lookupN3": ({"RP_LOOKUP_LDS": "1", "RP_LOOKUP_LDS_ABL": "4"}, 3),
        "lds-abl7/lookupN3": ({"RP_LOOKUP_LDS": "1", "RP_LOOKUP_LDS_ABL": "7"}, 3),
        # round 6: the wave-specialised kernel (NP producer : NC consumer waves a workgroup)
        "ws13/lookupN3": ({"RP_LOOKUP_WS": "1:3"}, 3),
        "ws26/lookupN3": ({"RP_LOOKUP_WS": "2:6"}, 3),
        "ws17/lookupN3": ({"RP_LOOKUP_WS": "1:7"}, 3),
        "ws412/lookupN3": ({"RP_LOOKUP_WS": "4:12"}, 3),
        "ws22/lookupN3": ({"RP_LOOKUP_WS": "2:2"}, 3),
        "ws115/lookupN3": ({"RP_LOOKUP_WS": "1:15"}, 3),
        "ws214/lookupN3": ({"RP_LOOKUP_WS": "2:14"}, 3),
        "ws412-abl1/lookupN3": ({"RP_LOOKUP_WS": "4:12", "RP_LOOKUP_WS_ABL": "1"}, 3),
        "ws412-abl2/lookupN3": ({"RP_LOOKUP_WS": "4:12", "RP_LOOKUP_WS_ABL": "2"}, 3),
        "ws13-g512/lookupN3": ({"RP_LOOKUP_WS": "1:3", "RP_LOOKUP_WS_GRID": "512"}, 3),
        "ws13-g2048/lookupN3": ({"RP_LOOKUP_WS": "1:3", "RP_LOOKUP_WS_GRID": "2048"}, 3),
    }
    if a.only:
        variants = {k: v for k, v in variants.items() if k in a.only.split(",")}
    knobs = ("RP_LOOKUP_HALF", "RP_LOOKUP_LEAN", "RP_LOOKUP_KPL", "RP_RING_LAYOUT", "RP_LOOKUP_ABLATE", "RP_RING_WIDE", "RP_LOOKUP_GRID", "RP_LOOKUP_OCC", "RP_LOOKUP_STG", "RP_LOOKUP_LH", "RP_LOOKUP_STGHS", "RP_LOOKUP_LDS", "RP_LOOKUP_LDS_GRID", "RP_LOOKUP_LDS_STG", "RP_LOOKUP_LDS_ABL", "RP_LOOKUP_WS", "RP_LOOKUP_WS_GRID", "RP_LOOKUP_WS_ABL")
    times = {k: [] for k in variants}
    digests = {}
    for r in range(a.rounds + 1):
        for name, (env, n) in variants.items():
            for kn in knobs:
                os.environ.pop(kn, None)
            os.environ.update(env)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            if n == 1:
                ring.lookup_dev(keys.data_ptr(), B, out.data_ptr(), 36, None, st.cuda_stream)
            else:
                ring.lookupn_dev(keys.data_ptr(), B, n, out.data_ptr(), None, 36, None, st.cuda_stream)
            e1.record(st)
            torch.cuda.synchronize()
            if r:
                times[name].append(e0.elapsed_time(e1))
            else:  # output digest per variant (lookupN(3) variants must agree)
                o = out[: B * n].long()
                digests[name] = int(torch.sum(o * (torch.arange(B * n, device="cuda") % 1009 + 1)).item())
    res = {}
    for name, t in times.items():
        med = float(np.median(t))
        res[name] = {"median_ms": med, "min_ms": float(np.min(t)), "Glookups_s": B / med / 1e6,
                     "alg_GBs": (48 if variants[name][1] == 3 else 40) * B / med / 1e6, "digest": digests[name]}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
