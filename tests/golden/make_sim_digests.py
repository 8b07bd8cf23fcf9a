"""Per-round digests of the gossip round model at the BASELINE configs' full sizes, computed by
the CPU oracle (oracle/orc_sim.c, pinned to the reference by tests/golden/sim_golden.json).

    python tests/golden/make_sim_digests.py [c4 c4s c5] [--threads T]

Writes tests/golden/sim_digests.json: for every case and round r, the SHA-256 of the vector of
all N membership checksums after round r (uint32 little-endian, 0 for nodes that are down), the
SHA-256 of every node's maxPiggybackCount, the cumulative stats (pings, ping-reqs, full syncs,
applied updates) and the first converged round (scenario-runner.js:152-170 + members that are
down faulty / members that left `leave` everywhere). The GPU tests (tests/test_sim_digests_gpu.py)
replay the same configs on the device and compare round by round.

Cases:
  c4   10,000 members, 1% (100) down from the start (Philox seed 11), suspicion 25 rounds
  c5   100,000 members, 1% (1,000) down, suspicion 25 rounds
  c4j  10,000 members, 1% down from the start; 100 running nodes crash at round 5; at round 45
       fresh processes for 50 of them and for 20 nodes down from the start join from join
       responses (mergeJoinResponses -> set(), RP_SIM_JOIN)
  c4s  10,000 members, 1% down from the start, then: 100 nodes leave at round 2
       (half-cluster-failure.js-style admin leaves), 100 running nodes crash at round 5, 50 of
       those come back at round 45 (they refute `faulty` and are answered with full syncs)
C5 takes ~10 minutes on 8 threads (~20 GB of host memory).
"""
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import pyoracle  # noqa: E402
from sim_configs import CASES, case_inputs  # noqa: E402


def run(name, threads):
    cfg = CASES[name]
    names, inc0, dead, events = case_inputs(cfg)
    t0 = time.time()
    sim = pyoracle.Sim(names, inc0, dead, seed=cfg["seed"], susp_rounds=cfg["susp"], now0=cfg["now0"],
                       events=events, threads=threads)
    print("%s: created in %.1f s" % (name, time.time() - t0), flush=True)
    out = {"name": name, "digests": [], "piggyback": [], "stats": [], "converged_round": None}
    last_ev = max((e[0] for e in events), default=0)  # convergence counts once every event ran
    for r in range(cfg["max_rounds"]):
        t = time.time()
        sim.step()
        ck = sim.checksums()
        out["digests"].append(hashlib.sha256(ck.astype("<u4").tobytes()).hexdigest())
        out["piggyback"].append(hashlib.sha256(sim.piggyback().astype("<u4").tobytes()).hexdigest())
        st = sim.stats()
        out["stats"].append([st["pings"], st["pingreqs"], st["fullsyncs"], st["applied"]])
        conv = sim.converged()
        if conv and out["converged_round"] is None and r >= last_ev:
            out["converged_round"] = r
        print("%s round %d: %.1f s %s conv=%s" % (name, r, time.time() - t, st, conv), flush=True)
        if out["converged_round"] is not None and r >= out["converged_round"] + cfg.get("after", 2):
            break
    out["rounds"] = len(out["digests"])
    return out


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    threads = 8
    if "--threads" in sys.argv:
        threads = int(sys.argv[sys.argv.index("--threads") + 1])
        args = [a for a in args if a != str(threads)]
    which = args or ["c4", "c4s", "c5"]
    path = os.path.join(HERE, "sim_digests.json")
    fixture = {"generator": "tests/golden/make_sim_digests.py (oracle/orc_sim.c)", "cases": {}}
    if os.path.exists(path):
        with open(path) as f:
            fixture = json.load(f)
    for name in which:
        fixture["cases"][name] = run(name, threads)
        with open(path, "w") as f:
            json.dump(fixture, f, indent=0, sort_keys=True)
        print("wrote", path, flush=True)


if __name__ == "__main__":
    main()
