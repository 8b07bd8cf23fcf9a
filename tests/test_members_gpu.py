"""GPU parity tests of the device membership merge + checksum through the C ABI.

Oracles: tests/golden/membership_golden.json (what the reference Membership did) and
oracle/orc_members.c (pinned against it in tests/test_oracle_membership.py). Bit-exact:
applied flags, rewritten updates, member table, checksum strings and checksums.
"""
import importlib.util
import os

import numpy as np
import pytest

import golden_util as gu

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STAT = {"alive": 0, "suspect": 1, "faulty": 2, "leave": 3}


def synth():
    spec = importlib.util.spec_from_file_location("rp_synth", os.path.join(REPO, "ringpop-node_amd", "synth.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def device_state(m, names):
    ex, st, inc = m.dump()
    ids = m.intern(names)
    return {a: (int(st[i]), int(inc[i])) for a, i in zip(names, ids) if ex[i]}


@pytest.mark.parametrize("fold", ["default", "bucket"])
@pytest.mark.parametrize("case_name", ["random", "fixture1332", "leave", "rules"])
def test_members_match_reference_goldens(gpu, case_name, fold, monkeypatch):
    """Every membership golden; "bucket" forces the large-batch bucket fold
    (RP_MEMBERS_BUCKET_FOLD=1) at the goldens' small batch sizes."""
    if fold == "bucket":
        monkeypatch.setenv("RP_MEMBERS_BUCKET_FOLD", "1")
    cases = gu.load("membership_golden.json")["cases"]
    sel = [c for c in cases if c["name"].startswith("rule/")] if case_name == "rules" else \
        [c for c in cases if c["name"] == case_name]
    for case in sel:
        m = gpu.Membership(whoami=case["local"])
        for op in case["ops"]:
            ch = op["changes"]
            ids = m.intern([c[0] for c in ch])
            app, nst, ninc, na = m.update_ids(ids, [STAT[c[1]] for c in ch], [c[2] for c in ch],
                                              now_ms=op.get("now", 0))
            got = [[i, gpu.STATUS_NAME[int(nst[i])], int(ninc[i])] for i in range(len(ch)) if app[i]]
            assert got == op["applied"], (case["name"], op.get("now"))
            assert na == len(got)
            assert m.checksum == op["checksum"], case["name"]
            if "members" in op:
                want = {w[0]: (STAT[w[1]], w[2]) for w in op["members"]}
                assert device_state(m, list(want)) == want
            if isinstance(op.get("checksumString"), str):
                assert m.generate_checksum_string() == op["checksumString"]


@pytest.mark.parametrize("fold", ["default", "bucket", "inline", "stream"])
def test_c3_merge_vs_oracle(gpu, orc, fold, monkeypatch):
    """C3 at full size: 100k members, 100k updates with 1% duplicated addresses (25 buckets of
    4,096 ids on the bucket path). Where each batch's checksum string is written (round 6,
    RP_MEMBERS_SIDE_BUILD): default, deferred into the next batch's fold launch from the row
    snapshot; "stream", on a build stream from the snapshot; "inline", right after the lengths."""
    if fold == "bucket":
        monkeypatch.setenv("RP_MEMBERS_BUCKET_FOLD", "1")
    if fold == "inline":
        monkeypatch.setenv("RP_MEMBERS_SIDE_BUILD", "0")
    if fold == "stream":
        monkeypatch.setenv("RP_MEMBERS_SIDE_BUILD", "1")
    S = synth()
    n = k = 100_000
    names, st0, inc0 = S.c3_members(n)
    m = gpu.Membership(whoami=names[0], capacity=n)
    o = orc.Members(names, local=names[0], join_seed=0)
    ids0 = np.asarray(m.intern(names), dtype=np.uint32)
    assert (ids0 == np.arange(n)).all()
    a0, _, _, na0 = m.update_ids(ids0, st0, inc0, now_ms=1)
    oa0, _, _, ona0 = o.update_ids(ids0, st0, inc0, False, 1)
    assert na0 == ona0 == n and (a0 == 2).all()
    assert m.checksum == o.checksum
    for batch in range(3):
        ids, us, ui = S.c3_updates(n, k, seed=7 + batch, base_inc=inc0)
        ga, gs, gi, gna = m.update_ids(ids, us, ui, now_ms=1434500000000 + batch)
        oa, os_, oi, ona = o.update_ids(ids, us, ui, False, 1434500000000 + batch)
        assert gna == ona
        assert np.array_equal(ga > 0, oa > 0)
        assert np.array_equal(gs[oa > 0], os_[oa > 0]) and np.array_equal(gi[oa > 0], oi[oa > 0])
        assert m.checksum == o.checksum
    ex, st, inc = m.dump()
    for i in range(0, n, 997):
        want = o.member(names[i])
        assert (gpu.STATUS_NAME[int(st[i])], int(inc[i])) == (want["status"], want["incarnationNumber"])
    assert m.generate_checksum_string() == o.checksum_string()


def test_update_dev_no_host_sync_path(gpu, orc):
    S = synth()
    n = 5000
    names, st0, inc0 = S.c3_members(n)
    m = gpu.Membership(whoami=names[1], capacity=n)
    dev_id = np.asarray(m.intern(names), dtype=np.uint32)  # whoami was interned first: ids != positions
    o = orc.Members(names, local=names[1])
    m.update_ids(dev_id, st0, inc0, now_ms=3)
    o.update_ids(np.arange(n), st0, inc0, False, 3)
    ids, us, ui = S.c3_updates(n, 20000, seed=11, base_inc=inc0)
    d_ids = torch.from_numpy(dev_id[ids].view(np.int32)).cuda()
    d_st = torch.from_numpy(us).cuda()
    d_inc = torch.from_numpy(ui).cuda()
    d_app = torch.empty(len(ids), dtype=torch.uint8, device="cuda")
    d_na = torch.zeros(1, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    m.update_dev(d_ids.data_ptr(), d_st.data_ptr(), d_inc.data_ptr(), len(ids), 77, d_app.data_ptr(), None, None,
                 d_na.data_ptr(), st)
    torch.cuda.synchronize()
    oa, _, _, ona = o.update_ids(ids, us, ui, False, 77)
    assert int(d_na.item()) == ona
    assert np.array_equal(d_app.cpu().numpy() > 0, oa > 0)
    assert m.checksum == o.checksum


def test_empty_and_checksum_null(gpu):
    m = gpu.Membership(whoami="127.0.0.1:3000")
    assert m.checksum is None
    app, _, _, na = m.update_ids([], [], [])
    assert na == 0 and m.checksum is None
    m.update([{"address": "127.0.0.1:3000", "status": "alive", "incarnationNumber": 5}])
    c1 = m.checksum
    assert c1 is not None
    assert m.update([{"address": "127.0.0.1:3000", "status": "alive", "incarnationNumber": 5}]) == []
    assert m.checksum == c1


def test_stash_set_matches_reference_golden(gpu):
    """isReady=false stash + Membership.set (index.js:208-247, merge.js:22-51) on the device,
    against the reference's recorded run (membership_golden.json 'stash-set')."""
    case = next(c for c in gu.load("membership_golden.json")["cases"] if c["name"] == "stash-set")
    m = gpu.Membership(whoami=case["local"])
    for op in case["ops"]:
        if op["type"] == "ready":
            m.set_ready(op["value"])
        elif op["type"] == "set":
            m.set()
        else:
            ch = op["changes"]
            ids = m.intern([c[0] for c in ch])
            app, nst, ninc, _ = m.update_ids(ids, [STAT[c[1]] for c in ch], [c[2] for c in ch],
                                             now_ms=op.get("now", 0), is_local=op.get("isLocal", False))
            got = [[i, gpu.STATUS_NAME[int(nst[i])], int(ninc[i])] for i in range(len(ch)) if app[i]]
            assert got == op["applied"]
        assert m.checksum == op["checksum"], op["type"]
        if "members" in op:
            want = {w[0]: (STAT[w[1]], w[2]) for w in op["members"]}
            assert device_state(m, list(want)) == want


def test_bootstrap_set_vs_oracle(gpu, orc):
    """The bulk bootstrap path at scale: 8 join responses x 20k members (overlapping addresses,
    incarnation ties, the local member inside), merged and set on the device; member table
    and checksum against the oracle, picks against mergeMembershipChangesets restated here."""
    S = synth()
    n, R, per = 30_000, 8, 20_000
    names = [S.c2_addr(i) for i in range(n)]
    rng = np.random.default_rng(5)
    ids = np.concatenate([rng.choice(n, size=per, replace=False) for _ in range(R)]).astype(np.uint32)
    st = rng.integers(0, 4, size=len(ids)).astype(np.uint8)
    inc = (1434401518824 + rng.integers(0, 3, size=len(ids))).astype(np.int64)
    m = gpu.Membership(whoami=names[0], capacity=n)
    assert m.intern(names) == list(range(n))
    o = orc.Members(names, local=names[0])
    m.set_ready(False)
    o.set_ready(False)
    for r in range(R):
        sl = slice(r * per, (r + 1) * per)
        m.update_ids(ids[sl], st[sl], inc[sl])
        o.update_ids(ids[sl], st[sl], inc[sl])
    picks = m.set()
    assert o.set() == len(picks)
    best, first = {}, []
    for j, a in enumerate(ids.tolist()):
        if a == 0:
            continue
        if a not in best:
            best[a] = j
            first.append(a)
        elif inc[best[a]] < inc[j]:
            best[a] = j
    assert picks == [(names[a], gpu.STATUS_NAME[int(st[best[a]])], int(inc[best[a]])) for a in first]
    assert m.checksum == o.checksum
    ex, dst, dinc = m.dump()
    for a in range(n):
        om = o.member(names[a])
        assert (om is None) == (not ex[a])
        if om:
            assert (gpu.STATUS_NAME[int(dst[a])], int(dinc[a])) == (om["status"], om["incarnationNumber"])


@pytest.mark.parametrize("nbatches,tail_noops", [(5, 0), (37, 3), (70, 0)])
def test_grouped_checksums_across_unread_batches(gpu, orc, nbatches, tail_noops):
    """Device batches whose checksums are never read in between: their strings wait in slots and
    are hashed side by side (groups of up to 64 per launch, on a side stream). A read after the
    last batch must equal the oracle's
    checksum after the same sequence — including when the last batches applied nothing (the
    checksum is then the last applying batch's), and across several full groups."""
    S = synth()
    n = k = 20_000
    names, st0, inc0 = S.c3_members(n)
    m = gpu.Membership(whoami=names[0], capacity=n)
    o = orc.Members(names, local=names[0], join_seed=0)
    ids0 = np.asarray(m.intern(names), dtype=np.uint32)
    m.update_ids(ids0, st0, inc0, now_ms=1)
    o.update_ids(ids0, st0, inc0, False, 1)
    stream = torch.cuda.current_stream()
    app = torch.empty(k, dtype=torch.uint8, device="cuda")
    na = torch.zeros(1, dtype=torch.int32, device="cuda")
    batches = [S.c3_updates(n, k, seed=50 + b, base_inc=inc0 + 3 * b) for b in range(nbatches)]
    batches += [batches[-1]] * tail_noops  # re-applying the last batch changes nothing... mostly
    for b, (ids, us, ui) in enumerate(batches):
        d = [torch.from_numpy(ids.view(np.int32)).cuda(), torch.from_numpy(us).cuda(), torch.from_numpy(ui).cuda()]
        m.update_dev(d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), k, 1434500000000 + b, app.data_ptr(),
                     None, None, na.data_ptr(), stream.cuda_stream)
        o.update_ids(ids, us, ui, False, 1434500000000 + b)
    torch.cuda.synchronize()
    assert m.checksum == o.checksum
    assert m.generate_checksum_string() == o.checksum_string()


def test_deferred_string_write_across_paths(gpu, orc, monkeypatch):
    """The deferred checksum-string write (round 6: batch b's string rides on batch b + 1's fold
    launch) across everything that must write it first instead: a batch on the bucket path, a
    batch on the sorted path, new members interned between batches (the writer reads the names'
    rank order), a Membership.set, an empty batch, and checksum reads; every batch's checksum
    against the oracle (read back from the per-batch history, rp_members_checksum_shard with one
    shard)."""
    import torch

    S = synth()
    n0, k = 3000, 2000
    names = [S.c2_addr(i) for i in range(n0 + 500)]
    m = gpu.Membership(whoami=names[0], capacity=n0)
    m.checksum_shard(1, 0, history_cap=64)
    o = orc.Members(names, local=names[0], join_seed=0)
    ids0 = np.asarray(m.intern(names[:n0]), dtype=np.uint32)
    st0 = np.zeros(n0, np.uint8)
    inc0 = np.full(n0, 100, np.int64)
    m.update_ids(ids0, st0, inc0, now_ms=1)
    o.update_ids(np.arange(n0), st0, inc0, False, 1)
    want = [o.checksum]
    stream = torch.cuda.current_stream().cuda_stream
    app = torch.empty(k, dtype=torch.uint8, device="cuda")
    na = torch.zeros(1, dtype=torch.int32, device="cuda")
    rng = np.random.default_rng(4)
    plan = ["g", "g", "bucket", "g", "sorted", "g", "intern", "g", "g", "read", "g", "empty", "g", "bucket",
            "bucket", "g", "g"]
    nn = n0
    keep = []
    for b, what in enumerate(plan):
        for e in ("RP_MEMBERS_BUCKET_FOLD", "RP_MEMBERS_SORTED_FOLD"):
            monkeypatch.delenv(e, raising=False)
        if what == "intern":
            new = names[nn:nn + 500]
            ids_new = np.asarray(m.intern(new), dtype=np.uint32)
            assert (ids_new == np.arange(nn, nn + 500)).all()
            nn += 500
            continue
        if what == "read":
            assert m.checksum == want[-1]
            continue
        if what == "bucket":
            monkeypatch.setenv("RP_MEMBERS_BUCKET_FOLD", "1")
        if what == "sorted":
            monkeypatch.setenv("RP_MEMBERS_SORTED_FOLD", "1")
        kk = 0 if what == "empty" else k
        ids = rng.integers(0, nn, size=kk).astype(np.uint32)
        us = rng.integers(0, 4, size=kk).astype(np.uint8)
        ui = (100 + b + rng.integers(0, 3, size=kk)).astype(np.int64)
        d = [torch.from_numpy(ids.view(np.int32)).cuda(), torch.from_numpy(us).cuda(), torch.from_numpy(ui).cuda()]
        keep.append(d)
        m.update_dev(d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), kk, 1434500000000 + b, app.data_ptr(),
                     None, None, na.data_ptr(), stream)
        if kk:
            o.update_ids(ids, us, ui, False, 1434500000000 + b)
            want.append(o.checksum)
    torch.cuda.synchronize()
    for e in ("RP_MEMBERS_BUCKET_FOLD", "RP_MEMBERS_SORTED_FOLD"):
        monkeypatch.delenv(e, raising=False)
    assert m.checksum == want[-1]
    h, a = m.checksum_history()
    assert len(h) == len(want) and a.all()  # (every batch here applies something)
    assert h.tolist() == want
    m.close()


@pytest.mark.parametrize("budget", [None, "3"], ids=["default-pool", "three-slots"])
def test_checksum_groups_wrap_with_reads(gpu, orc, budget, monkeypatch):
    """300 unread batches cycle through every slot group more than once (a group is rebuilt only
    after its previous chains finished), with checksum reads at scattered points in between: each
    read equals the oracle's checksum after the same prefix. RP_MEMBERS_CK_BYTES=3 leaves three
    one-string slots (groups of one)."""
    if budget:
        monkeypatch.setenv("RP_MEMBERS_CK_BYTES", str(int(budget) * 200_000))
    S = synth()
    n = k = 4000
    names, st0, inc0 = S.c3_members(n)
    m = gpu.Membership(whoami=names[0], capacity=n)
    o = orc.Members(names, local=names[0], join_seed=0)
    ids0 = np.asarray(m.intern(names), dtype=np.uint32)
    m.update_ids(ids0, st0, inc0, now_ms=1)
    o.update_ids(ids0, st0, inc0, False, 1)
    stream = torch.cuda.current_stream()
    app = torch.empty(k, dtype=torch.uint8, device="cuda")
    na = torch.zeros(1, dtype=torch.int32, device="cuda")
    reads = {17, 64, 65, 130, 199, 257}
    keep = []
    for b in range(300):
        ids, us, ui = S.c3_updates(n, k, seed=900 + b, base_inc=inc0 + 3 * b)
        d = [torch.from_numpy(ids.view(np.int32)).cuda(), torch.from_numpy(us).cuda(), torch.from_numpy(ui).cuda()]
        keep.append(d)
        m.update_dev(d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), k, 1434500000000 + b, app.data_ptr(),
                     None, None, na.data_ptr(), stream.cuda_stream)
        o.update_ids(ids, us, ui, False, 1434500000000 + b)
        if b in reads:
            assert m.checksum == o.checksum, b
    torch.cuda.synchronize()
    assert m.checksum == o.checksum


@pytest.mark.parametrize("sorted_fold", [False, True, "bucket"], ids=["grouped", "sorted", "bucket"])
def test_hot_addresses_take_the_overflow_fold(gpu, orc, sorted_fold, monkeypatch):
    """The grouped fold handles up to 16 changes per address in a batch; an address with more
    (here 17 and 60, next to addresses with exactly 16 and 15; later 3000 and 500 changes, so
    one address fills whole 1024-change chunks of k_fold_ovf and spans several) is folded by
    the gated overflow launch. Every batch - before, during and after the overflow - must match
    the oracle, and the grouped fold's per-address state must be clean again after an
    overflowing batch."""
    if sorted_fold == "bucket":
        monkeypatch.setenv("RP_MEMBERS_BUCKET_FOLD", "1")
    elif sorted_fold:
        monkeypatch.setenv("RP_MEMBERS_SORTED_FOLD", "1")
    S = synth()
    n = 3000
    names, st0, inc0 = S.c3_members(n)
    m = gpu.Membership(whoami=names[0], capacity=n)
    o = orc.Members(names, local=names[0], join_seed=0)
    ids0 = np.asarray(m.intern(names), dtype=np.uint32)
    m.update_ids(ids0, st0, inc0, now_ms=1)
    o.update_ids(ids0, st0, inc0, False, 1)
    rng = np.random.default_rng(5)
    for b, hot in enumerate([{7: 16, 8: 15}, {7: 17, 9: 60, 10: 16}, {11: 3}, {12: 40}, {13: 3000, 14: 500},
                             {13: 2}, {}]):
        ids, us, ui = S.c3_updates(n, 2000, seed=300 + b, base_inc=inc0 + 3 * b)
        ids, us, ui = list(ids), list(us), list(ui)
        for a, c in hot.items():
            for _ in range(c):
                p = int(rng.integers(0, len(ids) + 1))
                ids.insert(p, a)
                us.insert(p, int(rng.integers(0, 4)))
                ui.insert(p, int(inc0[a]) + 3 * b + int(rng.integers(-2, 3)))
        ids = np.asarray(ids, np.uint32)
        us = np.asarray(us, np.uint8)
        ui = np.asarray(ui, np.int64)
        ga, gs, gi, gna = m.update_ids(ids, us, ui, now_ms=1434500000000 + b)
        oa, os_, oi, ona = o.update_ids(ids, us, ui, False, 1434500000000 + b)
        assert gna == ona, b
        assert np.array_equal(ga > 0, oa > 0), b
        assert m.checksum == o.checksum, b
    assert m.generate_checksum_string() == o.checksum_string()


@pytest.mark.parametrize("applied_by", ["fold", "gather"])
def test_bucket_fold_repeats_overflow_and_large_batch(gpu, orc, monkeypatch, applied_by):
    """The bucket fold (batches of 2^19+ changes by default) against the oracle: a 2^20-change
    batch over 2^20 members (256 buckets of 4,096 ids; its applied flags, the status and
    incarnation of every change as rewritten by the local override, and the checksum), and a
    batch whose first four buckets hold 6,000 addresses with two changes each (12,000 repeated
    changes: more than a bucket's LDS list of 512, so the buckets' repeated addresses take the
    overflow fold); the local member's repeated suspect / faulty changes take the local
    override. applied_by "gather": the round-4 2-bit map and k_bk_gather (RP_BK_DIRECT=0) instead of
    the fold's direct stores."""
    if applied_by == "gather":
        monkeypatch.setenv("RP_BK_DIRECT", "0")
    S = synth()
    n = 1 << 20
    names, st0, inc0 = S.c3_members(n)
    m = gpu.Membership(whoami=names[0], capacity=n)
    o = orc.Members(names, local=names[0], join_seed=0)
    ids0 = np.asarray(m.intern(names), dtype=np.uint32)
    assert (ids0 == np.arange(n)).all()  # device ids are the oracle's positions
    m.update_ids(ids0, st0, inc0, now_ms=1)
    o.update_ids(ids0, st0, inc0, False, 1)
    ids, us, ui = S.c3_updates(n, n, seed=41, base_inc=inc0)
    ga, gs, gi, gna = m.update_ids(ids, us, ui, now_ms=1434500000007)
    oa, os_, oi, ona = o.update_ids(ids, us, ui, False, 1434500000007)
    assert gna == ona
    assert np.array_equal(ga > 0, oa > 0)
    assert np.array_equal(gs, os_) and np.array_equal(gi, oi)
    assert m.checksum == o.checksum
    monkeypatch.setenv("RP_MEMBERS_BUCKET_FOLD", "1")
    rng = np.random.default_rng(9)
    rep = rng.permutation(16384)[:6000].astype(np.uint32)
    ids = np.concatenate([rep, rng.integers(0, n, 20000).astype(np.uint32), rep[::-1], [0, 0, 0]]).astype(np.uint32)
    us = rng.integers(0, 4, len(ids)).astype(np.uint8)
    ui = (inc0[ids] + rng.integers(-1, 3, len(ids))).astype(np.int64)
    ga, gs, gi, gna = m.update_ids(ids, us, ui, now_ms=1434500000009)
    oa, os_, oi, ona = o.update_ids(ids, us, ui, False, 1434500000009)
    assert gna == ona
    assert np.array_equal(ga > 0, oa > 0)
    assert np.array_equal(gs, os_) and np.array_equal(gi, oi)
    assert m.checksum == o.checksum


def test_bucket_fold_bench_size(gpu, orc):
    """The bench's fold_large shape against the oracle: 2^22 members and a batch of 2^22 + 2^16
    changes (1,040 scatter tiles, so a fold lane walks three tile segments, not two; the 2^16
    ids past the table's size repeat an address, plus C3's 1 % repeats), in place, as bench.py
    runs it: applied flags, rewritten status / incarnation and the checksum."""
    import torch

    S = synth()
    n, k = 1 << 22, (1 << 22) + (1 << 16)
    names, st0, inc0 = S.c3_members(n)
    m = gpu.Membership(whoami=names[0], capacity=n)
    o = orc.Members(names, local=names[0], join_seed=0)
    ids0 = np.asarray(m.intern(names), dtype=np.uint32)
    m.update_ids(ids0, st0, inc0, now_ms=1)
    o.update_ids(ids0, st0, inc0, False, 1)
    ids, us, ui = S.c3_updates(n, k, seed=47, base_inc=inc0)
    now = 1434500000013
    oa, os_, oi, ona = o.update_ids(ids, us, ui, False, now)
    d_ids = torch.from_numpy(ids.view(np.int32)).cuda()
    d_st = torch.from_numpy(us.copy()).cuda()
    d_inc = torch.from_numpy(ui.copy()).cuda()
    d_app = torch.empty(k, dtype=torch.uint8, device="cuda")
    d_na = torch.zeros(1, dtype=torch.int32, device="cuda")
    m.update_dev(d_ids.data_ptr(), d_st.data_ptr(), d_inc.data_ptr(), k, now, d_app.data_ptr(), d_st.data_ptr(),
                 d_inc.data_ptr(), d_na.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert int(d_na.item()) == ona
    assert np.array_equal(d_app.cpu().numpy() > 0, oa > 0)
    assert np.array_equal(d_st.cpu().numpy(), os_) and np.array_equal(d_inc.cpu().numpy(), oi)
    assert m.checksum == o.checksum


@pytest.mark.parametrize("records", ["auto", "wide", "looped"])
def test_bucket_fold_wide_tiles_and_in_place_outputs(gpu, orc, monkeypatch, records):
    """The bucket fold's record formats (round 5) and outputs that alias the inputs, against the
    oracle. A 2^19-change batch over 2^19 members (128 scatter tiles): tiles 1 and 5 hold
    incarnations spanning more than 2^32 (12-B records there, 8-B records with a tile base
    elsewhere; records "wide": RP_BK_REC8=0, 12-B records everywhere; "looped": the scatter's
    A/B instance whose workgroups loop over tiles), and the local member has
    suspect / faulty changes that the local override rewrites. The status and incarnation
    outputs are the input arrays themselves, as the reference rewrites its update objects in
    place (member.js evaluateUpdate): after the call they must hold the oracle's outputs."""
    import torch

    if records == "wide":
        monkeypatch.setenv("RP_BK_REC8", "0")
    if records == "looped":  # the scatter's tile-loop instance (RP_BK_SGRID: 48 workgroups over 128 tiles)
        monkeypatch.setenv("RP_BK_SGRID", "48")
    S = synth()
    n = 1 << 19
    names, st0, inc0 = S.c3_members(n)
    m = gpu.Membership(whoami=names[0], capacity=n)
    o = orc.Members(names, local=names[0], join_seed=0)
    ids0 = np.asarray(m.intern(names), dtype=np.uint32)
    m.update_ids(ids0, st0, inc0, now_ms=1)
    o.update_ids(ids0, st0, inc0, False, 1)
    ids, us, ui = S.c3_updates(n, n, seed=43, base_inc=inc0)
    rng = np.random.default_rng(5)
    for t in (1, 5):  # a few far-future and far-past incarnations in two tiles
        at = t * 4096 + rng.permutation(4096)[:40]
        ui[at[:20]] += 1 << 33
        ui[at[20:]] = -(1 << 40) + rng.integers(0, 1000, 20)
    ids[[77, 4096 * 3 + 5, 4096 * 100 + 9]] = 0  # the local member
    us[[77, 4096 * 3 + 5, 4096 * 100 + 9]] = [1, 2, 1]
    ui[[77, 4096 * 3 + 5, 4096 * 100 + 9]] = inc0[0] + np.array([1, 2, 3])
    now = 1434500000011
    oa, os_, oi, ona = o.update_ids(ids, us, ui, False, now)
    d_ids = torch.from_numpy(ids.view(np.int32)).cuda()
    d_st = torch.from_numpy(us.copy()).cuda()
    d_inc = torch.from_numpy(ui.copy()).cuda()
    d_app = torch.empty(n, dtype=torch.uint8, device="cuda")
    d_na = torch.zeros(1, dtype=torch.int32, device="cuda")
    m.update_dev(d_ids.data_ptr(), d_st.data_ptr(), d_inc.data_ptr(), n, now, d_app.data_ptr(), d_st.data_ptr(),
                 d_inc.data_ptr(), d_na.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert int(d_na.item()) == ona
    assert np.array_equal(d_app.cpu().numpy() > 0, oa > 0)
    assert np.array_equal(d_st.cpu().numpy(), os_) and np.array_equal(d_inc.cpu().numpy(), oi)
    assert (oi[[77, 4096 * 3 + 5, 4096 * 100 + 9]] == now).all()  # the override ran
    assert m.checksum == o.checksum


def test_member_rows_incarnation_range(gpu, orc):
    """Member rows hold a 61-bit incarnation (8-B rows since round 5): the extremes of the range
    fold like any value against the oracle; one past it is refused by the host call (RP_EINVAL,
    nothing applied) and reported by the device call at the next sync (RP_EDEVICE)."""
    import torch

    names = ["10.9.0.%d:1" % i for i in range(8)]
    m = gpu.Membership(whoami=names[0], capacity=16)
    o = orc.Members(names, local=names[0], join_seed=0)
    ids = np.asarray(m.intern(names), dtype=np.uint32)
    lo, hi = -(1 << 60), (1 << 60) - 1
    for inc in ([lo] * 8, [hi - 1] * 8, [hi] * 8, [-5, 0, 1 << 53, lo + 1, hi, 7, -(1 << 59), 1 << 40]):
        st = np.array([0, 1, 2, 3, 0, 1, 2, 3], np.uint8)
        inc = np.asarray(inc, np.int64)
        ga, gs, gi, gna = m.update_ids(ids, st, inc, now_ms=1434500000000)
        oa, os_, oi, ona = o.update_ids(ids, st, inc, False, 1434500000000)
        assert gna == ona and np.array_equal(ga > 0, oa > 0)
        assert np.array_equal(gs, os_) and np.array_equal(gi, oi)
        assert m.checksum == o.checksum
    with pytest.raises(gpu.RingpopAmdError):
        m.update_ids(ids[:1], np.zeros(1, np.uint8), np.array([1 << 60], np.int64), now_ms=1)
    with pytest.raises(gpu.RingpopAmdError):
        m.update_ids(ids[:1], np.array([4], np.uint8), np.array([5], np.int64), now_ms=1)
    assert m.checksum == o.checksum  # nothing applied
    d_ids = torch.from_numpy(ids[1:2].view(np.int32)).cuda()
    d_st = torch.zeros(1, dtype=torch.uint8, device="cuda")
    d_inc = torch.full((1,), 1 << 61, dtype=torch.int64, device="cuda")
    m.update_dev(d_ids.data_ptr(), d_st.data_ptr(), d_inc.data_ptr(), 1, 2, None, None, None, None,
                 torch.cuda.current_stream().cuda_stream)
    with pytest.raises(gpu.RingpopAmdError):
        m.checksum
    m.close()


@pytest.mark.parametrize("path", ["grouped", "bucket", "set"])
def test_device_status_past_leave_reported(gpu, path, monkeypatch):
    """a status past leave (4) on a device call is not masked into alive..leave
    silently: update_dev (the grouped fold and the bucket fold, whose 8-B records keep 2 status
    bits) and set_dev report RP_EDEVICE at the handle's next sync, as an incarnation past 2^60
    does; a valid batch after it works again."""
    import torch

    if path == "bucket":
        monkeypatch.setenv("RP_MEMBERS_BUCKET_FOLD", "1")
    names = ["10.9.1.%d:1" % i for i in range(64)]
    m = gpu.Membership(whoami=names[0], capacity=64)
    ids = np.asarray(m.intern(names), dtype=np.uint32)
    m.update_ids(ids, np.zeros(64, np.uint8), np.full(64, 3, np.int64), now_ms=1)
    d_ids = torch.from_numpy(ids[1:9].view(np.int32)).cuda()
    st = np.array([0, 1, 2, 3, 4, 1, 0, 2], np.uint8)
    d_st = torch.from_numpy(st).cuda()
    d_inc = torch.full((8,), 9, dtype=torch.int64, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    if path == "set":
        m.set_ready(False)
        d_pick = torch.empty(9, dtype=torch.int32, device="cuda")
        gpu.check(gpu.lib().rp_members_set_dev(m._h, d_ids.data_ptr(), d_st.data_ptr(), d_inc.data_ptr(), 8,
                                               d_pick.data_ptr(), d_pick.data_ptr() + 32, s))
    else:
        m.update_dev(d_ids.data_ptr(), d_st.data_ptr(), d_inc.data_ptr(), 8, 2, None, None, None, None, s)
    with pytest.raises(gpu.RingpopAmdError, match="status past leave"):
        m.checksum
    m.set_ready(True)
    ga, _, _, gna = m.update_ids(ids[10:12], np.array([1, 2], np.uint8), np.array([7, 7], np.int64), now_ms=3)
    assert gna == 2 and m.checksum is not None
    m.close()
