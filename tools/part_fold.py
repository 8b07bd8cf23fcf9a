"""The id-partitioned 2^22 fold's per-rank work on one GPU (PartMembership's rank 0 alone):
rp_members_update_range_dev over the first 1/G of the buckets, for G = 1 (the whole update_dev),
2, 4, 8, alternating in one process, in place, HIP events per batch. What one rank of G on its
own GPU does (no collective on the fold's path), so it projects the leg's strong scaling.

    python tools/part_fold.py [--reps 12] [--log2 22]
"""
import argparse
import importlib.util
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=12)
    ap.add_argument("--log2", type=int, default=22)
    args = ap.parse_args()
    import torch
    rpa = _load("ringpop_node_amd", os.path.join(REPO, "ringpop-node_amd", "__init__.py"))
    S = _load("rp_synth", os.path.join(REPO, "ringpop-node_amd", "synth.py"))
    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream
    n = k = 1 << args.log2
    names = [S.c2_addr(i) for i in range(n)]
    inc0 = S.c3_members(n)[2]
    m = rpa.Membership(whoami=names[0], capacity=n)
    ids0 = np.asarray(m.intern(names), dtype=np.uint32)
    m.update_ids(ids0, np.zeros(n, np.uint8), inc0, now_ms=1)
    rpa.check(rpa.lib().rp_members_defer_checksum(m._h, 1))
    ids, us, ui = S.c3_updates(n, k, seed=300, base_inc=inc0)
    d_ids = torch.from_numpy(ids.view(np.int32)).cuda()
    d_st = torch.from_numpy(us).cuda()
    base_inc = torch.from_numpy(ui).cuda()
    app = torch.empty(k, dtype=torch.uint8, device="cuda")
    na = torch.zeros(1, dtype=torch.int32, device="cuda")
    G = [1, 2, 4, 8]
    res = {g: [] for g in G}
    lap = [0]

    def batch(g):
        # fresh incarnations every batch (3 more per batch: every change applies as a new batch would)
        lap[0] += 1
        inc = base_inc + 3 * lap[0]
        torch.cuda.synchronize()
        torch.cuda._sleep(2_000_000)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        if g == 1:
            m.update_dev(d_ids.data_ptr(), d_st.data_ptr(), inc.data_ptr(), k, 1434500000000 + lap[0], app.data_ptr(),
                         d_st.data_ptr(), inc.data_ptr(), na.data_ptr(), sp)
        else:
            m.update_range_dev(d_ids.data_ptr(), d_st.data_ptr(), inc.data_ptr(), k, 1434500000000 + lap[0], 0,
                               n // g, app.data_ptr(), d_st.data_ptr(), inc.data_ptr(), na.data_ptr(), sp)
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1), int(na.item())

    for g in G:
        batch(g)
    for r in range(args.reps):
        for g in G:
            ms, napp = batch(g)
            res[g].append((ms, napp))
    out = {"members": n, "updates": k, "reps": args.reps}
    for g in G:
        ms = [x[0] for x in res[g]]
        out["G%d" % g] = {"ms_p50": float(np.median(ms)), "ms_min": float(np.min(ms)), "ms_mean": float(np.mean(ms)),
                          "applied_last": res[g][-1][1]}
    print(json.dumps(out), flush=True)
    m.close()


if __name__ == "__main__":
    main()
