"""Per-kernel sums of the PMC passes of tools/pmc_wire.sh (counter_collection CSVs), for the
kernels whose name contains the given substrings. Usage: pmc_wire_summary.py DIR [substr ...]"""
import collections
import csv
import glob
import json
import sys

d = sys.argv[1]
subs = sys.argv[2:] or ["k_decode_wave"]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "")
        for s in subs:
            if s in k:
                key = s + ("<1280>" if "1280u" in k else "<2048>" if "2048u" in k else "")
                acc[key][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[key].add((f, r.get("Dispatch_Id")))
out = {k: {"dispatches_x_passes": len(disp[k]), **{c: v for c, v in sorted(acc[k].items())}} for k in acc}
for k, v in out.items():
    wc = v.get("SQ_WAVE_CYCLES", 0) or 1
    v["valu_active_per_wave_cycle"] = v.get("SQ_ACTIVE_INST_VALU", 0) / wc
    v["lds_active_per_wave_cycle"] = v.get("SQ_ACTIVE_INST_LDS", 0) / wc
    v["wait_any_per_wave_cycle"] = v.get("SQ_WAIT_ANY", 0) / wc
print(json.dumps(out, indent=1))
