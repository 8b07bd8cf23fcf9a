"""Debug helper: step the device simulator and the oracle side by side on a config of
tests/sim_configs.py (or a golden case) and report the first round where they differ: which
nodes, whether their views differ (protocol) or only their checksums (checksum engine)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import pyoracle  # noqa: E402
from conftest import load_pkg  # noqa: E402
from sim_configs import CASES, case_inputs  # noqa: E402

name = sys.argv[1]
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 10
G = int(sys.argv[3]) if len(sys.argv) > 3 else 0
cfg = dict(CASES[name])
names, inc0, dead, events = case_inputs(cfg)
rpa = load_pkg()
kw = dict(seed=cfg["seed"], suspicion_rounds=cfg["susp"], now0=cfg["now0"], events=events)
g = rpa.ShardedGossipSim(names, inc0, dead, G, **kw) if G else rpa.GossipSim(names, inc0, dead, **kw)
o = pyoracle.Sim(names, inc0, dead, seed=cfg["seed"], susp_rounds=cfg["susp"], now0=cfg["now0"], events=events,
                 threads=8)
ev_nodes = {}
for r, k, v in events:
    ev_nodes.setdefault(v, []).append((r, k))
for r in range(rounds):
    g.step()
    o.step()
    a, b = g.checksums(), o.checksums()
    sa, sb = g.stats(), o.stats()
    pa, pb = g.piggyback(), o.piggyback()
    bad = np.flatnonzero(a != b)
    print("round", r, "mismatch", len(bad), "stats", sa, sb, "piggy mismatch", int((pa != pb).sum()), flush=True)
    if len(bad) or sa != sb:
        for v in bad[:8]:
            gs, gi = g.view(int(v))
            os_, oi = o.view(int(v))
            dv = np.flatnonzero((gs != os_) | (gi != oi))
            print(" node", v, "events", ev_nodes.get(int(v)), "view diffs", len(dv),
                  [(int(x), int(gs[x]), int(os_[x]), int(gi[x]), int(oi[x]), ev_nodes.get(int(x))) for x in dv[:6]])
        break
