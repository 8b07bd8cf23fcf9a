"""Per-kernel summary (calls, total/avg/min/max ns) of a rocprofv3 --kernel-trace run, read
from its rocpd SQLite output (*_results.db) or a kernel_trace.csv; writes CSV to stdout."""
import csv
import sqlite3
import sys
from collections import defaultdict


def rows_from(path):
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        for name, dur in c.execute("select name, end - start from kernels"):
            yield name, int(dur)
    else:
        with open(path) as f:
            for r in csv.DictReader(f):
                yield r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"])


def main():
    acc = defaultdict(list)
    for p in sys.argv[1:]:
        for name, dur in rows_from(p):
            acc[name].append(dur)
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "Percentage"])
    tot = sum(sum(v) for v in acc.values()) or 1
    for name, v in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
        w.writerow([name, len(v), sum(v), sum(v) / len(v), min(v), max(v), "%.2f" % (100.0 * sum(v) / tot)])


if __name__ == "__main__":
    main()
