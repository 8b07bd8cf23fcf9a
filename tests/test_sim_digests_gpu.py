"""GPU parity of the simulator at the BASELINE configs' full sizes and a
10k-member scenario: every round, the SHA-256 of all N membership checksums and of every node's
maxPiggybackCount, the cumulative stats and the convergence round must equal the CPU oracle's
(tests/golden/sim_digests.json, made by tests/golden/make_sim_digests.py; the oracle itself is
pinned to the reference by tests/golden/sim_golden.json).

C5 runs once on one GPU (210 GB of view rows: 21 B per member per view) and once as 8 shard handles in one process
exchanging messages (the per-GPU layout of an 8-GPU run)."""
import hashlib

import numpy as np
import pytest

import golden_util as gu
from sim_configs import CASES, case_inputs

pytestmark = pytest.mark.gpu


def _replay(gpu, name, G=None):
    cfg = CASES[name]
    want = gu.load("sim_digests.json")["cases"][name]
    names, inc0, dead, events = case_inputs(cfg)
    kw = dict(seed=cfg["seed"], suspicion_rounds=cfg["susp"], now0=cfg["now0"], events=events)
    sim = gpu.ShardedGossipSim(names, inc0, dead, G, **kw) if G else gpu.GossipSim(names, inc0, dead, **kw)
    conv = None
    last_ev = max((e[0] for e in events), default=0)
    try:
        for r in range(want["rounds"]):
            sim.step()
            ck = sim.checksums()
            assert hashlib.sha256(ck.astype("<u4").tobytes()).hexdigest() == want["digests"][r], "round %d" % r
            pb = sim.piggyback()
            assert hashlib.sha256(pb.astype("<u4").tobytes()).hexdigest() == want["piggyback"][r], "round %d" % r
            st = sim.stats()
            assert [st["pings"], st["pingreqs"], st["fullsyncs"], st["applied"]] == want["stats"][r], "round %d" % r
            if conv is None and r >= last_ev and sim.converged():
                conv = r
        assert conv == want["converged_round"]
    finally:
        sim.close()


def test_c4_full_size(gpu):
    _replay(gpu, "c4")


def test_c4_scenario_full_size(gpu):
    _replay(gpu, "c4s")


def test_c4_scenario_sharded(gpu):
    _replay(gpu, "c4s", G=4)


def test_c4_join_full_size(gpu):
    """70 fresh processes bootstrapping into the 10k cluster from join responses."""
    _replay(gpu, "c4j")


def test_c4_join_sharded(gpu):
    """The same joins over 4 shard handles: responders and joiners on different shards."""
    _replay(gpu, "c4j", G=4)


def test_c5_full_size_one_gpu(gpu):
    _replay(gpu, "c5")


def test_c5_full_size_eight_shards(gpu):
    _replay(gpu, "c5", G=8)
