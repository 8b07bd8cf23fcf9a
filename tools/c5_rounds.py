"""C5 on one GPU round by round (instrument the p95 round): per round the wall
time (step + the convergence check that syncs it) and the views whose checksum chain ran that
round (the views_hashed counter: dirty views after the twin dedupe). With --no-twins the same
deterministic run hashes every dirty view (RP_SIM_TWINS=0 must be set by the caller), so the two
runs together give dirty views and distinct chains per round. Each chain is one serial farmhash
over the view's checksum string (base_len bytes ± its deviations).

    python tools/c5_rounds.py [--n 100000] [--label twins]
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
    ap.add_argument("--n", type=int, default=100_000)
    ap.add_argument("--label", default="default")
    ap.add_argument("--max-rounds", type=int, default=120)
    ap.add_argument("--shards", type=int, default=1, help="ShardedGossipSim in this process (one GPU)")
    args = ap.parse_args()
    import torch
    rpa = _load("ringpop_node_amd", os.path.join(REPO, "ringpop-node_amd", "__init__.py"))
    S = _load("rp_synth", os.path.join(REPO, "ringpop-node_amd", "synth.py"))
    n = args.n
    k = max(1, n // 100)
    names = [S.c2_addr(i) for i in range(n)]
    inc0 = S.c3_members(n)[2]
    dead = S.kill_set(n, k, 11)
    if args.shards > 1:
        sim = rpa.ShardedGossipSim(names, inc0, dead, args.shards, seed=11, suspicion_rounds=25)
    else:
        sim = rpa.GossipSim(names, inc0, dead, seed=11, suspicion_rounds=25)
    torch.cuda.synchronize()
    rows = []
    prev = sim.counters()["views_hashed"]
    for r in range(args.max_rounds):
        a = time.perf_counter()
        sim.step(1)
        c = sim.converged()
        ms = (time.perf_counter() - a) * 1e3
        vh = sim.counters()["views_hashed"]
        rows.append({"round": r, "ms": round(ms, 3), "views_hashed": vh - prev})
        prev = vh
        if c:
            break
    cnt = sim.counters()
    sim.close()
    ms = np.array([x["ms"] for x in rows])
    out = {"label": args.label, "n": n, "shards": args.shards, "rounds": len(rows), "base_len": cnt["base_len"],
           "chunks_per_chain": cnt["base_len"] // 20, "p50": float(np.percentile(ms, 50)),
           "p95": float(np.percentile(ms, 95)), "worst": int(ms.argmax()), "per_round": rows}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
