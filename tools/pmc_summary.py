"""Per-launch HBM traffic of the lookup kernel from tools/pmc_lookup.sh's rocprofv3 --pmc passes.

    python tools/pmc_summary.py gpurun_out/pmc_c > profiles/pmc_traffic.json

FETCH_SIZE on gfx950 reports 1/2 of a wide coalesced stream (MI355X_MICROARCH.md §HBM): the
hash-only ablation (same 36-B key stream, no table) calibrates that half, so traffic =
2 x (its FETCH) + (the kernel's FETCH - its FETCH) (the random table part, 64-B requests, taken as
reported; FETCH counts Infinity-Cache hits too) + WRITE_SIZE (exact for 16-B stores)."""
import collections
import csv
import glob
import json
import os
import sys


def main():
    d = sys.argv[1]
    res = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "k_lookupn_lean<8, 3, 4" in k or "k_lookupn_leanILi8ELi3ELi4E" in k:
                kk = "compact"
            elif "k_lookupn_probe<36, 2, 1>" in k:
                kk = "hashonly"
            elif "k_lookupn_fix_tiles" in k:
                kk = "fix"
            else:
                continue
            res[kk][r["Counter_Name"]].append(float(r["Counter_Value"]))
    avg = {kk: {c: sum(v) / len(v) for c, v in cs.items()} for kk, cs in res.items()}
    c, h, fx = avg["compact"], avg["hashonly"], avg.get("fix", {})
    keys = 1 << 26
    stream = 2 * h["FETCH_SIZE"] * 1024
    table = (c["FETCH_SIZE"] - h["FETCH_SIZE"]) * 1024
    writes = c["WRITE_SIZE"] * 1024
    fixb = (fx.get("FETCH_SIZE", 0) + fx.get("WRITE_SIZE", 0)) * 1024
    out = {
        "kernel": "k_lookupn_lean<8,3,4> (+ k_lookupn_fix_tiles)",
        "keys_per_launch": keys,
        "counters_per_launch": avg,
        "key_stream_bytes": stream,
        "table_bytes_beyond_l2": table,
        "write_bytes": writes,
        "fix_kernel_bytes": fixb,
        "lookupn_hbm_bytes_per_launch": stream + table + writes + fixb,
        "algorithmic_bytes_per_launch": 48 * keys,
        "l2_hit_rate": c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"]),
        "l1_to_l2_read_requests_per_key": c["TCP_TCC_READ_REQ_sum"] / keys,
        "method": "separate rocprofv3 --pmc passes (FETCH_SIZE | WRITE_SIZE | TCC_HIT_sum,TCC_MISS_sum | "
                  "TCC_EA0_RDREQ_sum | TCP_TCC_READ_REQ_sum) over tools/ab_lookup.py (tools/pmc_lookup.sh); "
                  "FETCH_SIZE of the key stream doubled per the gfx950 correction, calibrated with the hash-only "
                  "ablation kernel whose FETCH_SIZE is exactly half of the 2.42 GB of keys.",
    }
    # which kernel build the counters came from (bench.py reports it as traffic_measured_on)
    out["measured_on"] = os.environ.get("PMC_MEASURED_ON") or None
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
