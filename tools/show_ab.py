"""Print tools/ab_lookup.py JSON outputs as a table: python tools/show_ab.py f1.json [f2.json ...]"""
import json
import sys

for f in sys.argv[1:]:
    try:
        d = json.load(open(f))
    except Exception as e:  # noqa: BLE001
        print(f, e)
        continue
    print(f)
    for k, v in d.items():
        print("  %-26s %.3f ms %6.0f GB/s" % (k, v["median_ms"], v["alg_GBs"]))
