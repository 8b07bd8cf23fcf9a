"""C3 stream A/B in ONE process (bench.py's merge leg, checksummed batches), alternating
variants that differ only in environment read when a Membership handle is created or at each
update (the checksum pool and group sizes, RP_MEMBERS_*).

    python tools/c3_ab.py [--batches 1024] [--rounds 3] [--variants default,g256]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402

VARIANTS = {
    "default": {},
    "g256": {"RP_MEMBERS_GROUP_SLOTS": "256", "RP_MEMBERS_CK_BYTES": str(4 << 30)},
    "g192": {"RP_MEMBERS_GROUP_SLOTS": "192", "RP_MEMBERS_CK_BYTES": str(3 << 30)},
    "side": {"RP_MEMBERS_SIDE_BUILD": "1"},
    "fused": {"RP_MEMBERS_SIDE_BUILD": "2"},
    "fused-g512": {"RP_MEMBERS_SIDE_BUILD": "2", "RP_MEMBERS_GROUP_SLOTS": "512", "RP_MEMBERS_CK_BYTES": str(6 << 30)},
    "side-g512": {"RP_MEMBERS_SIDE_BUILD": "1", "RP_MEMBERS_GROUP_SLOTS": "512", "RP_MEMBERS_CK_BYTES": str(6 << 30)},
    "side-g256": {"RP_MEMBERS_SIDE_BUILD": "1", "RP_MEMBERS_GROUP_SLOTS": "256", "RP_MEMBERS_CK_BYTES": str(4 << 30)},
    "noside": {"RP_MEMBERS_SIDE_BUILD": "0"},
    "pad-g256": {"RP_HL_LDS_PAD": "65536", "RP_MEMBERS_GROUP_SLOTS": "256", "RP_MEMBERS_CK_BYTES": str(4 << 30)},
    "pad": {"RP_HL_LDS_PAD": "65536"},
    "nopack": {"RP_HL_PACK": "0"},
    "g512": {"RP_MEMBERS_GROUP_SLOTS": "512", "RP_MEMBERS_CK_BYTES": str(6 << 30)},
    "noside-g256": {"RP_MEMBERS_SIDE_BUILD": "0", "RP_MEMBERS_GROUP_SLOTS": "256", "RP_MEMBERS_CK_BYTES": str(4 << 30)},
}
KNOBS = ("RP_MEMBERS_GROUP_SLOTS", "RP_MEMBERS_CK_BYTES", "RP_MEMBERS_SIDE_BUILD", "RP_HL_LDS_PAD", "RP_HL_PACK")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=1024)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default="default,g256")
    a = ap.parse_args()
    import torch
    rpa = bench.load_pkg()
    names = a.variants.split(",")
    res = {v: [] for v in names}
    for r in range(a.rounds):
        for v in names:
            for k in KNOBS:
                os.environ.pop(k, None)
            os.environ.update(VARIANTS[v])
            out = bench.merge_bench(rpa, torch, 0, batches=a.batches, extras=False)
            res[v].append({"ms_per_batch": out["ms_per_batch"], "gpu_ms_per_batch": out["gpu_ms_per_batch"],
                           "checksum": out["checksum"]})
            print(v, r, json.dumps(res[v][-1]), flush=True)
            torch.cuda.empty_cache()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
