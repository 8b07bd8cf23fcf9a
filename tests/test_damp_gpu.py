"""GPU parity of the device damp scoring (rp_members_damp_*, rp_damp.h) through the C ABI.

Oracles: tests/golden/damp_golden.json (the reference Membership / Member run in node) and
oracle/orc_damp.c (pinned against it bit for bit in tests/test_oracle_damp.py).

Tolerance: none. The scores are IEEE doubles computed by the same operation sequence as the
engine (V8's fdlibm pow, Math.round half up, Math.max/min), so every dampScore,
lastUpdateDampScore and lastUpdateTimestamp must equal the reference's bit for bit, and the
'suppressLimitExceeded' events must come in the same order.
"""
import numpy as np
import pytest

import golden_util as gu

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
STAT = {"alive": 0, "suspect": 1, "faulty": 2, "leave": 3}


def run_case(rpa, case):
    m = rpa.Membership(whoami=case["local"])
    m.damp_configure(case["config"])
    for k, (op, o) in enumerate(zip(case["ops"], case["out"])):
        now = op["now"]
        sup = []
        if op["type"] == "ready":
            m.set_ready(op["value"])
        elif op["type"] == "set":
            m.set()
        elif op["type"] == "decay":
            m.damp_decay(now)
        else:
            ch = op["changes"]
            ids = m.intern([c[0] for c in ch])
            app, _, _, _ = m.update_ids(ids, [STAT[c[1]] for c in ch], [c[2] for c in ch], now_ms=now,
                                        is_local=op.get("isLocal", False))
            assert list(np.flatnonzero(app)) == o["applied"], (case["name"], k)
            if len(o["applied"]) or m.is_ready or op.get("isLocal"):
                _, exc = m.damp_last(len(ch))
                sup = [ch[i][0] for i in np.flatnonzero(exc)]
        assert sup == o["suppressed"], (case["name"], k)
        sc, ls, ts = m.damp_dump()
        ex, _, _ = m.dump()
        names = [x[0] for x in o["members"]]
        ids = m.intern(names)
        assert all(ex[i] for i in ids)
        got = [(a, float(sc[i]), float(ls[i]), int(ts[i])) for a, i in zip(names, ids)]
        want = [(x[0], float(x[1]), float(x[2]), x[3] or 0) for x in o["members"]]
        assert got == want, (case["name"], k, [(g, w) for g, w in zip(got, want) if g != w][:5])
    m.close()


@pytest.mark.parametrize("name", ["defaults", "flap", "half-life", "min-floor", "disabled", "fractional",
                                  "bootstrap", "wide"])
def test_damp_matches_reference_golden(gpu, name):
    case = next(c for c in gu.load("damp_golden.json")["cases"] if c["name"] == name)
    run_case(gpu, case)


def test_decay_sweep_vs_oracle_at_scale(gpu, orc):
    """The decayer over 200k members with random last scores / timestamps (0 = null included)
    equals the oracle's restatement bit for bit."""
    n = 200_000
    rng = np.random.default_rng(5)
    names = ["10.%d.%d.%d:3000" % (i >> 16, (i >> 8) & 255, i & 255) for i in range(n)]
    m = gpu.Membership(whoami=names[0], capacity=n)
    cfg = {"dampScoringPenalty": 377, "dampScoringHalfLife": 45, "dampScoringMin": 3}
    m.damp_configure(cfg)
    ids = m.intern(names)
    t0 = 1434401518824
    # every member created, then 24 batches of applied penalties (refuted with a higher
    # incarnation each time) at spread-out times
    m.update_ids(ids, np.zeros(n, np.uint8), np.full(n, 5, np.int64), now_ms=t0)
    for r in range(24):
        sel = rng.choice(n, n // 8, replace=False)
        m.update_ids(np.asarray(ids)[sel], np.zeros(len(sel), np.uint8), np.full(len(sel), 6 + r, np.int64),
                     now_ms=t0 + 2500 * (r + 1) + int(rng.integers(0, 2000)))
    sc, ls, ts = m.damp_dump()
    now = t0 + 75_000
    m.damp_decay(now)
    got, _, _ = m.damp_dump()
    ex = np.ones(n, np.uint8)
    want = np.empty(n, np.float64)
    c = orc.damp_cfg(cfg)
    orc.damp_decay_all(c, ex, ls.copy(), ts.copy(), now, want)
    assert np.array_equal(got.view(np.uint64), want.view(np.uint64))
    assert (ts == 0).sum() > 0 and len(np.unique(got)) > 50
    m.close()


def test_damp_errors_are_loud(gpu):
    m = gpu.Membership(whoami="a:1")
    with pytest.raises(gpu.RingpopAmdError):
        m.damp_decay(5)
    with pytest.raises(gpu.RingpopAmdError):
        m.damp_configure({"dampScoringHalfLife": 0})
    m.close()
