"""GPU parity tests of the gossip round simulator (librpamd rp_sim_*) against the reference
goldens (tests/golden/sim_golden.json: the reference modules driven through the round model)
and against the CPU oracle (oracle/orc_sim.c) on larger seeded cases: every live node's
checksum after every round, final views, stats, convergence. Bit-exact."""
import importlib.util
import os

import numpy as np
import pytest

import golden_util as gu

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STAT = {"alive": 0, "suspect": 1, "faulty": 2, "leave": 3}


def synth():
    spec = importlib.util.spec_from_file_location("rp_synth", os.path.join(REPO, "ringpop-node_amd", "synth.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


CASES = [c["name"] for c in gu.load("sim_golden.json")["cases"]]


def _golden_sim(gpu, case, G=None):
    S = synth()
    n = case["n"]
    names = [S.c2_addr(i) for i in range(n)]
    args = (names, S.c3_members(n)[2], np.array(case["dead"], dtype=np.uint8))
    kw = dict(seed=case["seed"], suspicion_rounds=case["suspRounds"], now0=case["now0"], events=case["events"])
    return names, (gpu.ShardedGossipSim(*args, G, **kw) if G else gpu.GossipSim(*args, **kw))


@pytest.mark.parametrize("case_name", CASES)
def test_sim_matches_reference_goldens(gpu, case_name):
    """Every node's checksum and maxPiggybackCount after every round, the full syncs sent and the
    final member tables equal what the reference modules produced (tests/golden/ref_sim.js),
    including the scenario cases: admin leaves, crashes mid-run, revivals answered with a full
    sync that refute `faulty`, and a ring size crossing a power of ten (maxPiggyback 45 -> 30)."""
    case = next(c for c in gu.load("sim_golden.json")["cases"] if c["name"] == case_name)
    names, sim = _golden_sim(gpu, case)
    for r, want in enumerate(case["checksums"]):
        sim.step()
        assert sim.checksums().tolist() == want, "round %d" % r
        assert sim.piggyback().tolist() == case["maxPiggyback"][r], "round %d" % r
    assert sim.stats()["fullsyncs"] == case["fullSyncs"]
    for v, view in zip(case["views"], case["finalViews"]):
        st, inc = sim.view(v)
        got = {names[i]: (int(st[i]), int(inc[i])) for i in range(case["n"])}
        assert got == {a: (STAT[s], i) for a, s, i in view}
    sim.close()


@pytest.mark.parametrize("mode", ["scan", "xcap3", "ck_pc", "ck_block"])
def test_sim_d1_paths_match_reference_goldens(gpu, monkeypatch, mode):
    """Phase D1's two ways of drawing ping-req helpers give the reference's helpers: the members-
    array scan (RP_SIM_OPOS_BYTES=0: no inverse permutation) and the mixed run where views with
    more than 3 non-candidates scan while the others select through the sorted non-candidate
    positions (RP_SIM_D1_XCAP=3). The default run (the goldens above) selects everywhere. The
    senders' checksums (default: k_ck_pair, the lane-pair chains) also run through k_ck_pc
    (RP_SIM_D1_CK=pc) and a workgroup per sender (blockck)."""
    if mode == "scan":
        monkeypatch.setenv("RP_SIM_OPOS_BYTES", "0")
    elif mode == "xcap3":
        monkeypatch.setenv("RP_SIM_D1_XCAP", "3")
    else:
        monkeypatch.setenv("RP_SIM_D1_CK", "pc" if mode == "ck_pc" else "blockck")
    for case in gu.load("sim_golden.json")["cases"]:
        names, sim = _golden_sim(gpu, case)
        for r, want in enumerate(case["checksums"]):
            sim.step()
            assert sim.checksums().tolist() == want, (case["name"], r)
        assert sim.stats()["fullsyncs"] == case["fullSyncs"]
        sim.close()


@pytest.mark.parametrize("kernel", ["pc", "lanes", "pc32", "pair"])
def test_sim_twins_match_reference_goldens(gpu, monkeypatch, kernel):
    """Every scenario golden with the twin-view pass forced on (RP_SIM_TWINS=1) on both chain
    kernels: late rounds have many equal views, each takes its representative's checksum. The
    fingerprints block_apply keeps per view (joins recompute theirs) are checked against a scan of
    every dirty view's rows each refresh (RP_SIM_TWIN_VERIFY=1: a difference raises)."""
    monkeypatch.setenv("RP_SIM_TWINS", "1")
    monkeypatch.setenv("RP_SIM_TWIN_VERIFY", "1")
    monkeypatch.setenv("RP_SIM_CK", kernel)
    for case in gu.load("sim_golden.json")["cases"]:
        names, sim = _golden_sim(gpu, case)
        for r, want in enumerate(case["checksums"]):
            sim.step()
            assert sim.checksums().tolist() == want, (case["name"], r)
        sim.close()


@pytest.mark.parametrize("case_name", ["n40-leave", "n24-revive", "n64-half-leave"])
def test_sharded_sim_matches_reference_goldens(gpu, case_name):
    """The same scenario goldens through the sharded path (3 shard handles, message exchanges
    between them): a leave runs on the shard that owns the node, down flags on every shard."""
    case = next(c for c in gu.load("sim_golden.json")["cases"] if c["name"] == case_name)
    _, sim = _golden_sim(gpu, case, G=3)
    for r, want in enumerate(case["checksums"]):
        sim.step()
        assert sim.checksums().tolist() == want, "round %d" % r
        assert sim.piggyback().tolist() == case["maxPiggyback"][r], "round %d" % r
    assert sim.stats()["fullsyncs"] == case["fullSyncs"]
    sim.close()


@pytest.mark.parametrize("n,k,seed,susp", [(500, 5, 3, 25), (1000, 10, 11, 25), (777, 40, 9, 7)])
def test_sim_vs_oracle(gpu, orc, n, k, seed, susp):
    S = synth()
    names = [S.c2_addr(i) for i in range(n)]
    inc0 = S.c3_members(n)[2]
    dead = S.kill_set(n, k, seed)
    g = gpu.GossipSim(names, inc0, dead, seed=seed, suspicion_rounds=susp)
    o = orc.Sim(names, inc0, dead, seed=seed, susp_rounds=susp, now0=1434401518824 + 10 ** 9)
    conv_g = conv_o = None
    for r in range(60):
        g.step()
        o.step()
        assert np.array_equal(g.checksums(), o.checksums()), "round %d" % r
        if conv_o is None and o.converged():
            conv_o = r
        if conv_g is None and g.converged():
            conv_g = r
    assert conv_g == conv_o is not None
    assert g.stats() == o.stats()
    for v in (0, n // 2, n - 1):
        if dead[v]:
            continue
        gs, gi = g.view(v)
        os_, oi = o.view(v)
        assert np.array_equal(gs, os_) and np.array_equal(gi, oi)


@pytest.mark.parametrize("twins", ["0", "1"])
@pytest.mark.parametrize("kernel", ["pc", "lanes", "pc3", "pc32", "pair", "lanes-p1", "pc32-p1", "lanes+p1"])
def test_sim_checksum_kernels_vs_oracle(gpu, orc, monkeypatch, kernel, twins):
    """Both lane-checksum kernels (k_ck_pc: chain wave + producer waves; k_ck_lanes: one wave per
    64 nodes), forced through RP_SIM_CK, against the oracle on a case with many deviations; with
    and without the twin-view pass (equal views hash once, compacted view lists). "-p1": each lane
    walks its own view's pass 1 (RP_SIM_PASS1=0) instead of k_pass1's wave per view, "+p1" the
    other way round (k_ck_lanes defaults to its own walks)."""
    if kernel[-3:] in ("-p1", "+p1"):
        monkeypatch.setenv("RP_SIM_PASS1", "0" if kernel[-3] == "-" else "1")
        kernel = kernel[:-3]
    monkeypatch.setenv("RP_SIM_CK", kernel)
    monkeypatch.setenv("RP_SIM_TWINS", twins)
    monkeypatch.setenv("RP_SIM_TWIN_VERIFY", twins)
    S = synth()
    n, k, seed, susp = 900, 60, 5, 6
    names = [S.c2_addr(i) for i in range(n)]
    inc0 = S.c3_members(n)[2]
    dead = S.kill_set(n, k, seed)
    g = gpu.GossipSim(names, inc0, dead, seed=seed, suspicion_rounds=susp)
    o = orc.Sim(names, inc0, dead, seed=seed, susp_rounds=susp, now0=1434401518824 + 10 ** 9)
    for r in range(30):
        g.step()
        o.step()
        assert np.array_equal(g.checksums(), o.checksums()), "round %d" % r


def test_sim_dlist_overflow_falls_back_to_bitmap(gpu, orc, monkeypatch):
    """RP_SIM_DLIST_BYTES small enough that every view's deviated-piece list overflows: the lane
    checksums must take the bitmap-scan fallback and still match the oracle every round."""
    monkeypatch.setenv("RP_SIM_DLIST_BYTES", str(16 * 600 * 4))  # 4 pieces per view
    S = synth()
    n, k, seed, susp = 600, 30, 4, 5
    names = [S.c2_addr(i) for i in range(n)]
    inc0 = S.c3_members(n)[2]
    dead = S.kill_set(n, k, seed)
    ev = [(3, "leave", 5), (20, "revive", int(np.flatnonzero(dead)[0]))]
    g = gpu.GossipSim(names, inc0, dead, seed=seed, suspicion_rounds=susp, events=ev)
    o = orc.Sim(names, inc0, dead, seed=seed, susp_rounds=susp, now0=1434401518824 + 10 ** 9, events=ev)
    for r in range(40):
        g.step()
        o.step()
        assert np.array_equal(g.checksums(), o.checksums()), "round %d" % r
    assert g.stats() == o.stats()
    g.close()


def test_sim_capacity_overflow_is_loud(gpu, monkeypatch):
    """A dissemination list past its capacity is reported, never silently truncated."""
    monkeypatch.setenv("RP_SIM_CAP", "3")
    S = synth()
    n = 200
    g = gpu.GossipSim([S.c2_addr(i) for i in range(n)], S.c3_members(n)[2], S.kill_set(n, 20, 3), seed=3,
                      suspicion_rounds=3)
    with pytest.raises(gpu.RingpopAmdError, match="capacity"):
        for _ in range(30):
            g.step()
    g.close()


@pytest.mark.parametrize("case_name", ["n30-join", "n70-join"])
@pytest.mark.parametrize("G", [2, 3])
def test_sharded_sim_join_matches_reference_goldens(gpu, case_name, G):
    """Join events on the sharded path: every shard exports the rows of the responders it owns
    (rp_sim_join_export), the buffers are combined (rp_sim_join_exchange_local) and the joiner's
    shard builds its view (rp_sim_join_import). Same checksums and piggyback counts every round
    as the reference goldens."""
    case = next(c for c in gu.load("sim_golden.json")["cases"] if c["name"] == case_name)
    _, sim = _golden_sim(gpu, case, G=G)
    for r, want in enumerate(case["checksums"]):
        sim.step()
        assert sim.checksums().tolist() == want, "round %d" % r
        assert sim.piggyback().tolist() == case["maxPiggyback"][r], "round %d" % r
    assert sim.stats()["fullsyncs"] == case["fullSyncs"]
    sim.close()


def test_sharded_join_without_exchange_is_refused(gpu):
    """Stepping shard handles directly (no join export / import) into a join event is refused
    loudly instead of being approximated."""
    case = next(c for c in gu.load("sim_golden.json")["cases"] if c["name"] == "n30-join")
    _, sim = _golden_sim(gpu, case, G=2)
    with pytest.raises(gpu.RingpopAmdError, match="join"):
        for _ in range(25):
            for k in range(gpu.SIM_STAGES):
                for s in sim.shards:
                    s.stage(k)
                if k < gpu.SIM_STAGES - 1:
                    gpu.check(gpu.lib().rp_sim_exchange_local(sim._arr, sim.G))
    sim.close()


@pytest.mark.parametrize("case_name", ["n30-join", "n70-join"])
def test_sharded_join_twins_verified(gpu, monkeypatch, case_name):
    """Joins rewrite the joiner's rows wholesale; its kept twin fingerprint is recomputed from the
    rows (k_vfp_view) and checked by RP_SIM_TWIN_VERIFY with the twin pass forced on."""
    monkeypatch.setenv("RP_SIM_TWINS", "1")
    monkeypatch.setenv("RP_SIM_TWIN_VERIFY", "1")
    test_sharded_sim_join_matches_reference_goldens(gpu, case_name, 2)


def test_sim_with_early_refresh_matches_reference_goldens(gpu, monkeypatch):
    """RP_SIM_EARLY=1: the stage-2 refresh beside the D1 chains (off by default);
    the goldens must hold either way."""
    monkeypatch.setenv("RP_SIM_EARLY", "1")
    test_sim_matches_reference_goldens(gpu, "n24-revive")
    test_sim_matches_reference_goldens(gpu, "n30-join")
