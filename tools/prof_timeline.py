"""Per-kernel and per-stream timeline summary of a rocprofv3 kernel-trace database (rocpd SQLite,
the default output of `rocprofv3 --kernel-trace -d DIR -o NAME`).

    python tools/prof_timeline.py DB [--match k_link,k_fold_fast,...] [--last N]

Prints, per kernel name: count, mean / median duration; per queue (stream): busy time, span
and the busy fraction over the span of the last N dispatches of the matched kernels.
"""
import argparse
import collections
import re
import sqlite3

import numpy as np


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--match", default="")
    ap.add_argument("--last", type=int, default=0)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    names = {r[0]: re.sub(r"^(void )?(rp::)?(\(anonymous namespace\)::)?", "", r[1]) for r in c.execute("select id, kernel_name from rocpd_info_kernel_symbol")}
    rows = list(c.execute("select kernel_id, queue_id, stream_id, start, end from rocpd_kernel_dispatch order by start"))
    pats = [p for p in a.match.split(",") if p]
    if pats:
        rows = [r for r in rows if any(p in names[r[0]] for p in pats)]
    if a.last:
        rows = rows[-a.last:]
    per = collections.defaultdict(list)
    for k, q, s, t0, t1 in rows:
        per[names[k].split("(")[0]].append((t1 - t0) / 1e3)
    print("%-60s %6s %9s %9s" % ("kernel", "n", "mean_us", "med_us"))
    for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        print("%-60s %6d %9.2f %9.2f" % (k[:60], len(v), np.mean(v), np.median(v)))
    byq = collections.defaultdict(list)
    for k, q, s, t0, t1 in rows:
        byq[(q, s)].append((t0, t1))
    t_all0 = min(r[3] for r in rows)
    t_all1 = max(r[4] for r in rows)
    print("span %.1f us over %d dispatches" % ((t_all1 - t_all0) / 1e3, len(rows)))
    for (q, s), iv in byq.items():
        iv.sort()
        busy, cur0, cur1 = 0, iv[0][0], iv[0][1]
        for t0, t1 in iv[1:]:
            if t0 > cur1:
                busy += cur1 - cur0
                cur0, cur1 = t0, t1
            else:
                cur1 = max(cur1, t1)
        busy += cur1 - cur0
        print("queue %s stream %s: %d dispatches, busy %.1f us (%.0f %% of the span)"
              % (q, s, len(iv), busy / 1e3, 100.0 * busy / (t_all1 - t_all0)))


if __name__ == "__main__":
    main()
