"""Runs the device gossip simulator at C5 shape (or n) for a fixed number of rounds, for PMC and
trace passes over the checksum kernels. Usage: python tools/sim_c5_probe.py [n] [rounds] [kill_pct]"""
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 12
kp = int(sys.argv[3]) if len(sys.argv) > 3 else 1
torch.cuda.set_device(0)
rpa = bench.load_pkg()
S = bench._synth()
k = max(1, n * kp // 100)
names = [S.c2_addr(i) for i in range(n)]
sim = rpa.GossipSim(names, S.c3_members(n)[2], S.kill_set(n, k, 11), seed=11, suspicion_rounds=25, device=0)
for r in range(rounds):
    t = time.perf_counter()
    sim.step(1)
    sim.converged()
    print("round %d %.1f ms" % (r, (time.perf_counter() - t) * 1e3), flush=True)
sim.close()
