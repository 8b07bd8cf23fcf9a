"""SQ counters of the simulator's checksum kernels (tools/pmc_ck.sh passes) summed per kernel.

    python tools/pmc_ck_summary.py LABEL=DIR [LABEL=DIR ...]

Prints {label: {kernel: {counter: sum over dispatches}}} as JSON."""
import collections
import csv
import glob
import json
import os
import re
import sys


def short(name):
    m = re.search(r"(k_[A-Za-z0-9_]+)", name)
    return m.group(1) if m else name[:40]


def summarise(d):
    res = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            res[short(r["Kernel_Name"])][r["Counter_Name"]] += float(r["Counter_Value"])
    return {k: dict(v) for k, v in res.items()}


def main():
    out = {}
    for a in sys.argv[1:]:
        label, d = a.split("=", 1)
        out[label] = summarise(d)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
