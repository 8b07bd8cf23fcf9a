"""Kernel statistics from a rocprofv3 results database (run_results.db; rocprofv3 without
--output-format csv writes sqlite): per kernel name and grid size, calls / mean / min / max µs.

    python tools/prof_db.py gpurun_out/prof_x/run_results.db [--csv out.csv] [--match substr]"""
import argparse
import sqlite3
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv")
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    gx = "grid_size_x" if "grid_size_x" in cols else ("grid_size" if "grid_size" in cols else None)
    q = "select name, %s, start, end from kernels" % (gx or "0")
    by = {}
    for name, grid, s, e in c.execute(q):
        if a.match and a.match not in name:
            continue
        by.setdefault((name, grid), []).append((e - s) / 1e3)
    rows = sorted(by.items(), key=lambda kv: -sum(kv[1]))
    lines = ["Name,Grid,Calls,TotalUs,AverageUs,MedianUs,MinUs,MaxUs"]
    for (name, grid), d in rows:
        lines.append('"%s",%s,%d,%.1f,%.2f,%.2f,%.2f,%.2f' % (name.replace('"', "'"), grid, len(d), sum(d),
                                                          sum(d) / len(d), statistics.median(d), min(d), max(d)))
    txt = "\n".join(lines)
    if a.csv:
        open(a.csv, "w").write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main()
