"""Membership fold A/B on the GPU box (RP_AMD_LIB selects the library build).

    python tools/merge_fold_ab.py [--label L] [--reps N] [--only c3,c3ck,big]

Times, with HIP events on the launch stream:
  c3    the C3 fold alone (100k members, 100k-update batches, checksum deferred), per batch;
  c3ck  C3 with the checksum string built per batch (chains grouped as in bench.py), per batch;
  big   the fold at 2^22 members x 2^22 updates (checksum deferred), per batch.
Prints one JSON line. Used under rocprofv3 --pmc by tools/pmc_merge.sh (fewer reps there).
"""
import argparse
import importlib.util
import json
import os
import sys
import time

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
    ap.add_argument("--label", default=os.environ.get("RP_AMD_LIB", "librpamd.so"))
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default="c3,c3ck,big")
    ap.add_argument("--big-log2", type=int, default=22)
    ap.add_argument("--inplace", action="store_true", help="status / incarnation outputs alias the inputs")
    args = ap.parse_args()
    only = set(args.only.split(","))
    import torch
    rpa = _load("ringpop_node_amd", os.path.join(REPO, "ringpop-node_amd", "__init__.py"))
    S = _load("rp_synth", os.path.join(REPO, "ringpop-node_amd", "synth.py"))
    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream
    out = {"label": args.label}

    def run(n, k, nsets, reps, defer, seed0):
        names = [S.c2_addr(i) for i in range(n)]
        inc0 = S.c3_members(n)[2]
        m = rpa.Membership(whoami=names[0], capacity=n)
        ids0 = np.asarray(m.intern(names), dtype=np.uint32)
        m.update_ids(ids0, np.zeros(n, np.uint8), inc0, now_ms=1)
        sets = []
        for q in range(nsets):
            ids, us, ui = S.c3_updates(n, k, seed=seed0 + q, base_inc=inc0 + 3 * q)
            sets.append((torch.from_numpy(ids.view(np.int32)).cuda(), torch.from_numpy(us).cuda(),
                         torch.from_numpy(ui).cuda()))
        app = torch.empty(k, dtype=torch.uint8, device="cuda")
        nst = torch.empty(k, dtype=torch.uint8, device="cuda")
        ninc = torch.empty(k, dtype=torch.int64, device="cuda")
        na = torch.zeros(1, dtype=torch.int32, device="cuda")
        if defer:
            rpa.check(rpa.lib().rp_members_defer_checksum(m._h, 1))

        # every batch's incarnations prepared before the timed region (set b % nsets, raised by
        # 3 * nsets per lap so each batch is fresh against the table)
        incs = [sets[b % nsets][2] + 3 * nsets * (b // nsets) for b in range(reps + 2)]

        def one(b):
            d = sets[b % nsets]
            os_, oi = (d[1], incs[b]) if args.inplace else (nst, ninc)
            m.update_dev(d[0].data_ptr(), d[1].data_ptr(), incs[b].data_ptr(), k, 1434500000000 + b, app.data_ptr(),
                         os_.data_ptr(), oi.data_ptr(), na.data_ptr(), sp)
            return None

        keep = [one(b) for b in range(2)]
        torch.cuda.synchronize()
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
        t0 = time.perf_counter()
        for b in range(reps):
            evs[b][0].record(stream)
            keep.append(one(2 + b))
            evs[b][1].record(stream)
        if not defer:
            _ = m.checksum
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) * 1e3 / reps
        ms = [a.elapsed_time(c) for a, c in evs]
        napp = int(na.item())
        m.close()
        return {"members": n, "updates": k, "ms_mean": float(np.mean(ms)), "ms_min": float(np.min(ms)),
                "ms_p50": float(np.median(ms)), "wall_ms_per_batch": wall, "applied_last": napp,
                "GBps_49B": 49 * k / (float(np.mean(ms)) * 1e-3) / 1e9}

    if "c3" in only:
        out["c3"] = run(100_000, 100_000, 16, args.reps, True, 100)
    if "c3ck" in only:
        out["c3ck"] = run(100_000, 100_000, 16, max(args.reps, 8), False, 100)
    if "big" in only:
        nb = 1 << args.big_log2
        out["big"] = run(nb, nb, 3, max(2, args.reps // 3), True, 300)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
