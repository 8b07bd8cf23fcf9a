"""CPU tests: the gossip round-model oracle (oracle/orc_sim.c) reproduces, round by round,
every live node's membership checksum and maxPiggybackCount that the REFERENCE modules produced
when driven through the same round model (tests/golden/ref_sim.js), plus the full syncs they
sent and final member tables — for the kill-only cases and the scenario cases (leave, crash
mid-run, revive with refutation and full sync, ring size crossing a power of ten, fresh
processes joining from join responses)."""
import importlib.util
import os

import numpy as np
import pytest

import golden_util as gu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STAT = {"alive": 0, "suspect": 1, "faulty": 2, "leave": 3}
CASES = [c["name"] for c in gu.load("sim_golden.json")["cases"]]


def synth():
    spec = importlib.util.spec_from_file_location("rp_synth", os.path.join(REPO, "ringpop-node_amd", "synth.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.mark.parametrize("threads", [1, 4])
@pytest.mark.parametrize("case_name", CASES)
def test_sim_oracle_matches_reference(orc, case_name, threads):
    S = synth()
    case = next(c for c in gu.load("sim_golden.json")["cases"] if c["name"] == case_name)
    n = case["n"]
    names = [S.c2_addr(i) for i in range(n)]
    inc0 = S.c3_members(n)[2]
    sim = orc.Sim(names, inc0, np.array(case["dead"], dtype=np.uint8), seed=case["seed"],
                  susp_rounds=case["suspRounds"], now0=case["now0"], events=case["events"], threads=threads)
    for r, want in enumerate(case["checksums"]):
        sim.step()
        assert sim.checksums().tolist() == want, "round %d" % r
        assert sim.piggyback().tolist() == case["maxPiggyback"][r], "round %d" % r
    assert sim.stats()["fullsyncs"] == case["fullSyncs"]
    for v, view in zip(case["views"], case["finalViews"]):
        st, inc = sim.view(v)
        got = {names[i]: (int(st[i]), int(inc[i])) for i in range(n)}
        assert got == {a: (STAT[s], i) for a, s, i in view}


def test_sim_oracle_windowed_order_matches_whole(orc, monkeypatch):
    """The members-array window (used when N^2 order entries exceed ORC_SIM_ORDER_BYTES, as at
    C5) regenerates exactly the whole-array walk, including reshuffles on wrap."""
    S = synth()
    n, k, seed = 300, 30, 2
    names = [S.c2_addr(i) for i in range(n)]
    inc0 = S.c3_members(n)[2]
    dead = S.kill_set(n, k, seed)
    ev = [(40, "revive", int(np.flatnonzero(dead)[0])), (5, "leave", 7), (60, "join", int(np.flatnonzero(dead)[1])),
          (90, "join", 7), (90, "join", 11)]
    whole = orc.Sim(names, inc0, dead, seed=seed, susp_rounds=3, events=ev)
    monkeypatch.setenv("ORC_SIM_ORDER_BYTES", "100")
    win = orc.Sim(names, inc0, dead, seed=seed, susp_rounds=3, events=ev, threads=3)
    for r in range(360):  # > N rounds: every iterator wraps and reshuffles
        whole.step()
        win.step()
        assert np.array_equal(whole.checksums(), win.checksums()), "round %d" % r
    assert whole.stats() == win.stats()
