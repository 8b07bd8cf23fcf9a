"""CPU tests: the numpy Philox of ringpop-node_amd/synth.py equals the oracle's C Philox and the
Random123 known answers; the C3 generator has the documented shape."""
import importlib.util
import os

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def synth():
    spec = importlib.util.spec_from_file_location("rp_synth", os.path.join(REPO, "ringpop-node_amd", "synth.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_numpy_philox_matches_oracle_and_kat(orc):
    S = synth()
    out = S.philox4x32_10([0, 0xFFFFFFFF], [0, 0xFFFFFFFF], [0, 0xFFFFFFFF], [0, 0xFFFFFFFF], 0, 0)
    assert [int(x[0]) for x in out] == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    r = S.stream(7, S.TAG_UPDATE, 64, start=1000)
    for q in (0, 5, 63):
        assert [int(x[q]) for x in r] == orc.philox([1000 + q, 0, 0, 0], [7, S.TAG_UPDATE])


def test_c3_generator_shape():
    S = synth()
    names, st, inc = S.c3_members(1000)
    assert len(set(names)) == 1000 and (st == 0).all()
    assert ((inc >= S.BASE_INC) & (inc < S.BASE_INC + 10 ** 8)).all()
    ids, us, ui = S.c3_updates(1000, 5000)
    assert ids.max() < 1000
    frac = np.bincount(us, minlength=4) / len(us)
    assert abs(frac[0] - 0.70) < 0.03 and abs(frac[3] - 0.05) < 0.02
    d = ui - inc[ids]
    assert set(np.unique(d)) <= {-1, 0, 1}
