"""The simulator configs of SURVEY §8d at full size (C4, C5) plus a 10k scenario, shared by the
digest generator (tests/golden/make_sim_digests.py, CPU oracle) and the GPU tests that replay
them (tests/test_sim_digests_gpu.py). Inputs are deterministic (ringpop-node_amd/synth.py)."""
import importlib.util
import os

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NOW0 = 1434401518824 + 10 ** 9


def synth():
    spec = importlib.util.spec_from_file_location("rp_synth", os.path.join(REPO, "ringpop-node_amd", "synth.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


CASES = {
    "c4": {"n": 10_000, "kill_pct": 1, "seed": 11, "susp": 25, "now0": NOW0, "max_rounds": 80},
    "c5": {"n": 100_000, "kill_pct": 1, "seed": 11, "susp": 25, "now0": NOW0, "max_rounds": 80},
    "c4s": {"n": 10_000, "kill_pct": 1, "seed": 11, "susp": 25, "now0": NOW0, "max_rounds": 140, "scenario": True,
            "after": 4},
    # 100 running nodes crash at round 5; at round 45 fresh processes for 50 of them, and for 20
    # of the nodes down from the start, bootstrap back in from join responses
    "c4j": {"n": 10_000, "kill_pct": 1, "seed": 11, "susp": 25, "now0": NOW0, "max_rounds": 140, "scenario": "join",
            "after": 4},
}


def case_inputs(cfg):
    """(names, inc0, dead, events) of a config."""
    S = synth()
    n = cfg["n"]
    k = max(1, n * cfg["kill_pct"] // 100)
    names = [S.c2_addr(i) for i in range(n)]
    inc0 = S.c3_members(n)[2]
    dead = S.kill_set(n, k, cfg["seed"])
    events = []
    if cfg.get("scenario") == "join":
        live = np.flatnonzero(dead == 0)
        r = np.random.default_rng(cfg["seed"] + 1)
        crashed = r.permutation(live)[:100]
        events += [(5, "kill", int(v)) for v in sorted(crashed)]
        events += [(45, "join", int(v)) for v in sorted(crashed[:50])]
        events += [(45, "join", int(v)) for v in np.flatnonzero(dead)[:20]]
    elif cfg.get("scenario"):
        live = np.flatnonzero(dead == 0)
        r = np.random.default_rng(cfg["seed"])
        pick = r.permutation(live)
        leavers, crashed = pick[:100], pick[100:200]
        events += [(2, "leave", int(v)) for v in sorted(leavers)]
        events += [(5, "kill", int(v)) for v in sorted(crashed)]
        events += [(45, "revive", int(v)) for v in sorted(crashed[:50])]
    return names, inc0, dead, events
