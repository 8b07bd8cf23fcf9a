"""C3 merge per-batch timeline. On the GPU box, under rocprofv3 --kernel-trace:

    python tools/c3_timeline.py run [batches]        # the C3 leg alone (bench.merge_bench, no extras)
    python tools/c3_timeline.py show results.db      # per-batch kernel sequence of the steady state

`show` cuts the kernel trace at each k_link launch (one per update batch) and prints, for a
few steady-state batches, every kernel with its queue, start offset from the batch's k_link,
duration and the idle gap before it on its queue, then the mean batch period, the busy time per
queue and the mean gap: a period well above the main queue's busy time is launch (host) bound."""
import os
import sqlite3
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(batches):
    sys.path.insert(0, REPO)
    import bench
    import torch
    rpa = bench.load_pkg()
    torch.cuda.set_device(0)
    out = bench.merge_bench(rpa, torch, 0, batches=batches, extras=False)
    print(out["updates_per_s"] / 1e6, "M updates/s", out["ms_per_batch"], "ms/batch")


def show(db):
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    qcol = "queue_id" if "queue_id" in cols else ("stream_id" if "stream_id" in cols else None)
    rows = list(c.execute("select name, start, end, %s from kernels order by start" % (qcol or "0")))
    short = [(n.replace("rp::(anonymous namespace)::", "").replace("void ", "").split("(")[0][:40], s, e, q)
             for n, s, e, q in rows]
    links = [i for i, r in enumerate(short) if r[0] == "k_link"]
    if len(links) < 8:
        print("fewer than 8 k_link launches")
        return
    mid = links[len(links) // 2: len(links) // 2 + 4]
    last_end = {}
    for i, r in enumerate(short):
        if i == mid[0]:
            break
        last_end[r[3]] = r[2]
    for a, b in zip(mid, mid[1:]):
        t0 = short[a][1]
        print("--- batch at k_link #%d" % links.index(a))
        for n, s, e, q in short[a:b]:
            gap = (s - last_end.get(q, s)) / 1e3
            last_end[q] = e
            print("  q%-3s %-40s +%8.2f us  dur %7.2f  gap %6.2f" % (q, n, (s - t0) / 1e3, (e - s) / 1e3, gap))
    per = [(short[b][1] - short[a][1]) / 1e3 for a, b in zip(links[5:-5], links[6:-4])]
    print("batch period: mean %.2f us, median %.2f" % (statistics.mean(per), statistics.median(per)))
    busy = {}
    span0, span1 = short[links[5]][1], short[links[-5]][1]
    for n, s, e, q in short:
        if span0 <= s < span1:
            busy[q] = busy.get(q, 0) + (e - s)
    nb = len(links) - 10
    for q, v in busy.items():
        print("queue %s busy %.2f us per batch" % (q, v / 1e3 / nb))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(int(sys.argv[2]) if len(sys.argv) > 2 else 256)
    else:
        show(sys.argv[2])
