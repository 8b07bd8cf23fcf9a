"""Per-shard cost of the C5 simulator on ONE GPU: N members split into G shard handles in one
process (ShardedGossipSim; the shards run one after another on the same device, so each
kernel's duration under rocprofv3 is what one GPU of a G-GPU run spends on its shard).
Usage: python tools/shard_probe.py N G rounds"""
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402

n, G, rounds = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
torch.cuda.set_device(0)
rpa = bench.load_pkg()
S = bench._synth()
k = max(1, n // 100)
names = [S.c2_addr(i) for i in range(n)]
sim = rpa.ShardedGossipSim(names, S.c3_members(n)[2], S.kill_set(n, k, 11), G, seed=11, suspicion_rounds=25)
t0 = time.perf_counter()
conv = None
for r in range(rounds):
    sim.step()
    if conv is None and sim.converged():
        conv = r
    print("round %d %.1f s" % (r, time.perf_counter() - t0), flush=True)
torch.cuda.synchronize()
print({"n": n, "shards": G, "rounds": rounds, "converged_round": conv,
       "wall_s_per_round_all_shards": (time.perf_counter() - t0) / rounds})
sim.close()
