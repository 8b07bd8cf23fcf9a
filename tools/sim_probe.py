"""Times the device gossip simulator at a given size (C4 scaling probe): rounds until
convergence, per-round wall time. Usage: python tools/sim_probe.py N [kill_pct] [max_rounds]"""
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402

n = int(sys.argv[1])
kp = int(sys.argv[2]) if len(sys.argv) > 2 else 1
mr = int(sys.argv[3]) if len(sys.argv) > 3 else 300
torch.cuda.set_device(0)
rpa = bench.load_pkg()
t0 = time.perf_counter()
print(bench.sim_bench(rpa, 0, n=n, kill_pct=kp, max_rounds=mr, max_seconds=200), flush=True)
print("total %.1f s" % (time.perf_counter() - t0))
