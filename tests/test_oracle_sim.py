"""CPU tests: the gossip round-model oracle (oracle/orc_sim.c) reproduces, round by round,
every live node's membership checksum that the REFERENCE modules produced when driven through
the same round model (tests/golden/ref_sim.js), plus final member tables."""
import importlib.util
import os

import numpy as np
import pytest

import golden_util as gu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STAT = {"alive": 0, "suspect": 1, "faulty": 2, "leave": 3}


def synth():
    spec = importlib.util.spec_from_file_location("rp_synth", os.path.join(REPO, "ringpop-node_amd", "synth.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.mark.parametrize("case_name", ["n16k1", "n64k2", "n128k3-susp4", "n200k10"])
def test_sim_oracle_matches_reference(orc, case_name):
    S = synth()
    case = next(c for c in gu.load("sim_golden.json")["cases"] if c["name"] == case_name)
    n = case["n"]
    names = [S.c2_addr(i) for i in range(n)]
    inc0 = S.c3_members(n)[2]
    sim = orc.Sim(names, inc0, np.array(case["dead"], dtype=np.uint8), seed=case["seed"],
                  susp_rounds=case["suspRounds"], now0=case["now0"])
    for r, want in enumerate(case["checksums"]):
        sim.step()
        assert sim.checksums().tolist() == want, "round %d" % r
    for v, view in zip(case["views"], case["finalViews"]):
        st, inc = sim.view(v)
        got = {names[i]: (int(st[i]), int(inc[i])) for i in range(n)}
        assert got == {a: (STAT[s], i) for a, s, i in view}
