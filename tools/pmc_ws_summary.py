"""PMC passes of the lookupN kernels (tools/sessions/r06ay.sh) averaged per kernel instance.

    python tools/pmc_ws_summary.py DIR

Prints {kernel<template args>: {counter: mean per dispatch, "dispatches": n, "ms": mean duration}}
as JSON (one entry per template instance, so the lean kernel and each k_lookupn_ws<NP, NC, ABL>
stay apart)."""
import collections
import csv
import glob
import json
import os
import re
import sys


def short(name):
    m = re.search(r"(k_[A-Za-z0-9_]+(<[^>]*>)?)", name)
    return m.group(1) if m else name[:40]


def main():
    d = sys.argv[1]
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.defaultdict(lambda: collections.defaultdict(set))
    dur = collections.defaultdict(dict)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if not k.startswith(("k_lookupn_lean", "k_lookupn_ws")):
                continue
            key = (f, r["Dispatch_Id"])
            tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
            cnt[k][r["Counter_Name"]].add(key)
            dur[k][key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    out = {}
    for k in tot:
        out[k] = {c: tot[k][c] / len(cnt[k][c]) for c in tot[k]}
        out[k]["dispatches"] = len(dur[k])
        out[k]["ms"] = sum(dur[k].values()) / max(1, len(dur[k]))
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
