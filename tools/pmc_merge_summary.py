"""Per-launch counters of the membership fold kernels from tools/pmc_merge.sh passes.

    python tools/pmc_merge_summary.py gpurun_out/pmc_merge_new [gpurun_out/pmc_merge_r02 ...]

Groups dispatches by (kernel, grid size): the C3 batches (100k updates) and the 2^22 batches
launch different grids. HBM bytes per launch = 2 x FETCH_SIZE (gfx950: FETCH_SIZE reports half
of a 128-B request, MI355X_MICROARCH.md §HBM; for scattered 16-B row accesses this is an upper
bound) + WRITE_SIZE, both in KiB in the counters. Per update = / the batch's updates."""
import collections
import csv
import glob
import json
import os
import re
import sys


def short(name):
    m = re.match(r"(?:void )?(?:rp::)?(?:\(anonymous namespace\)::)?([A-Za-z0-9_]+)(<[^(]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:60]


def summarise(d):
    res = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = (short(r["Kernel_Name"]), int(r.get("Grid_Size", r.get("Grid_Size_X", 0)) or 0))
            res[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for (kn, grid), cs in sorted(res.items()):
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        e = {"grid_threads": grid, "dispatches": max(len(v) for v in cs.values()), "counters": avg}
        if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
            e["hbm_bytes"] = (2 * avg["FETCH_SIZE"] + avg["WRITE_SIZE"]) * 1024
        if "TCC_HIT_sum" in avg:
            t = avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"]
            e["l2_hit_rate"] = avg["TCC_HIT_sum"] / t if t else None
        out["%s@%d" % (kn, grid)] = e
    return out


def main():
    print(json.dumps({os.path.basename(d.rstrip("/")): summarise(d) for d in sys.argv[1:]}, indent=1))


if __name__ == "__main__":
    main()
