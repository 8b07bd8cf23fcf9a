"""Membership merge on G GPUs as batch-strided replicas (DistMembership):
every rank folds every batch on its own replica; rank g checksums batches b % G == g. The
per-batch checksums gathered from the ranks, and every replica's table, must equal one
single-GPU Membership folding the same stream with a checksum after every batch (the
reference's Membership.update computes one per applied batch, lib/membership/index.js:306-309).
Ranks share the box's one GPU here (gloo transport); an 8-GPU node runs the same code."""
import importlib.util
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _reference(gpu, n, k, nbatch):
    """The single-GPU sequence: checksum read after every batch (host path: one per batch)."""
    S = _load("rp_synth", os.path.join(REPO, "ringpop-node_amd", "synth.py"))
    W = _load("dist_merge_worker", os.path.join(REPO, "tests", "workers", "dist_merge_worker.py"))
    names, _, inc0 = S.c3_members(n)
    m = gpu.Membership(whoami=names[0], capacity=n)
    m.intern(names)
    cks = []
    for b, (ids, us, ui) in enumerate(W.batches(S, n, k, nbatch, inc0)):
        m.update_ids(ids, us, ui, now_ms=1434500000000 + b)
        cks.append(m.checksum)
    ex, st, inc = m.dump()
    m.close()
    return cks, ex, st, inc


@pytest.mark.parametrize("G,mode", [(2, ""), (3, ""), (2, "each")])
def test_dist_membership_matches_single_gpu(gpu, tmp_path, G, mode):
    """mode "each": every rank reads latest_checksum() after every batch (the value of a batch
    another rank hashed) through a 2-entry device history that each read drains; only the entries
    since the previous read are gathered. The .checksum property refuses on G > 1 ranks (a read on
    one rank alone would hang a collective)."""
    n, k, nbatch = 6000, 5000, 7
    out = str(tmp_path / "merge.npz")
    port = _free_port()
    worker = os.path.join(REPO, "tests", "workers", "dist_merge_worker.py")
    procs = []
    for r in range(G):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK="0", WORLD_SIZE=str(G), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, worker, str(n), str(k), str(nbatch), out, "gloo", mode],
                                      env=env))
    assert [p.wait(timeout=100) for p in procs] == [0] * G
    d = np.load(out)
    cks, ex, st, inc = _reference(gpu, n, k, nbatch)
    assert [int(c) for c in d["checksums"]] == cks
    if mode == "each":
        assert [int(c) for c in d["reads"]] == cks
    assert np.array_equal(d["ex"], ex) and np.array_equal(d["st"], st) and np.array_equal(d["inc"], inc)


def test_checksum_history_full_refuses_before_applying(gpu):
    """A batch whose history entry would not fit history_cap fails with RP_ESTATE and applies
    nothing (the table and the handle's pending state are as before); after a drain the stream
    goes on and every recorded value equals a plain handle's."""
    S = _load("rp_synth", os.path.join(REPO, "ringpop-node_amd", "synth.py"))
    n = k = 2000
    names, _, inc0 = S.c3_members(n)
    a = gpu.Membership(whoami=names[0], capacity=n)
    b = gpu.Membership(whoami=names[0], capacity=n)
    a.intern(names)
    b.intern(names)
    a.checksum_shard(1, 0, 3)
    with pytest.raises(gpu.RingpopAmdError):  # a deferred batch would record no entry
        gpu.check(gpu.lib().rp_members_defer_checksum(a._h, 1))
    want = []
    for i in range(5):
        ids, us, ui = S.c3_updates(n, k, seed=900 + i, base_inc=inc0 + 3 * (i // 2))
        if i == 3:
            before = a.dump()
            with pytest.raises(gpu.RingpopAmdError, match="history full"):
                a.update_ids(ids, us, ui, now_ms=1 + i)
            after = a.dump()
            assert all(np.array_equal(x, y) for x, y in zip(before, after))
            h, _ = a.checksum_history()
            assert len(h) == 3
            gpu.check(gpu.lib().rp_members_checksum_history_drain(a._h, 2))
        a.update_ids(ids, us, ui, now_ms=1 + i)
        b.update_ids(ids, us, ui, now_ms=1 + i)
        want.append(b.checksum)
    h, app = a.checksum_history()  # batch 2 (kept by the drain of two), 3, 4
    assert list(app) == [1, 1, 1] and [int(x) for x in h] == want[2:5]


def test_checksum_history_single_handle(gpu):
    """One handle with nshards = 1 records every batch's checksum: equal to reading it after
    each batch, across slot groups (more batches than a group holds)."""
    S = _load("rp_synth", os.path.join(REPO, "ringpop-node_amd", "synth.py"))
    n = k = 3000
    names, _, inc0 = S.c3_members(n)
    a = gpu.Membership(whoami=names[0], capacity=n)
    b = gpu.Membership(whoami=names[0], capacity=n)
    a.intern(names)
    b.intern(names)
    a.checksum_shard(1, 0, 1000)
    want = []
    for i in range(300):
        ids, us, ui = S.c3_updates(n, k, seed=500 + i, base_inc=inc0 + 3 * (i // 2))
        a.update_ids(ids, us, ui, now_ms=1 + i)
        b.update_ids(ids, us, ui, now_ms=1 + i)
        want.append(b.checksum)
    h, app = a.checksum_history()
    got, cur = [], None
    for x, y in zip(h, app):
        cur = int(x) if y else cur
        got.append(cur)
    assert got == want


def _reference_part(gpu, n, k, nbatch):
    """The single-GPU sequence for the partitioned run: checksum and applied flags after every batch."""
    S = _load("rp_synth", os.path.join(REPO, "ringpop-node_amd", "synth.py"))
    W = _load("part_merge_worker", os.path.join(REPO, "tests", "workers", "part_merge_worker.py"))
    names, _, inc0 = S.c3_members(n)
    m = gpu.Membership(whoami=names[0], capacity=n)
    m.intern(names)
    cks, apps = [], []
    for b, (ids, us, ui) in enumerate(W.batches(S, n, k, nbatch, inc0)):
        app, _, _, _ = m.update_ids(ids, us, ui, now_ms=1434500000000 + b)
        apps.append(app.copy())
        cks.append(m.checksum)
    ex, st, inc = m.dump()
    m.close()
    return cks, np.concatenate(apps), ex, st, inc


@pytest.mark.parametrize("G,n", [(2, 4 * 4096 + 1234), (3, 4 * 4096 + 1234), (3, 6000)])
def test_part_membership_matches_single_gpu(gpu, tmp_path, G, n):
    """The merge partitioned by member id (PartMembership): every rank folds the
    changes of its own ids (whole 4,096-id buckets) from the same batch stream, and the rows are
    all-gathered for the checksum after every batch. Per-batch checksums, every change's applied
    flag (from the rank owning its id; no rank writes another's) and the final table equal one
    single-GPU Membership's. A table of 5 buckets gives ranks 3+2 or 2+2+1 of them; one of 2
    buckets over 3 ranks leaves the last rank none (its updates fold nothing). The last batch sends
    300 changes each to an address of the first and of the last rank (past the bucket fold's LDS
    list: the overflow fold)."""
    k, nbatch = 9000, 5
    out = str(tmp_path / "part.npz")
    port = _free_port()
    worker = os.path.join(REPO, "tests", "workers", "part_merge_worker.py")
    procs = []
    for r in range(G):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK="0", WORLD_SIZE=str(G), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, worker, str(n), str(k), str(nbatch), out, "gloo"], env=env))
    assert [p.wait(timeout=100) for p in procs] == [0] * G
    d = np.load(out)
    cks, apps, ex, st, inc = _reference_part(gpu, n, k, nbatch)
    assert [int(c) for c in d["checksums"]] == cks
    assert np.array_equal(d["applied"], apps)
    assert np.array_equal(d["ex"], ex) and np.array_equal(d["st"], st) and np.array_equal(d["inc"], inc)


def test_update_range_matches_whole_update(gpu):
    """rp_members_update_range_dev over complementary ranges, one after the other on one handle,
    equals one update_dev of the whole batch (2^19 changes: the bucket path either way) on
    another: same table, checksum and applied flags; a range that is not whole buckets is refused."""
    S = _load("rp_synth", os.path.join(REPO, "ringpop-node_amd", "synth.py"))
    n = 1 << 18
    names, st0, inc0 = S.c3_members(n)
    a = gpu.Membership(whoami=names[0], capacity=n)
    b = gpu.Membership(whoami=names[0], capacity=n)
    a.intern(names)
    b.intern(names)
    for m in (a, b):
        m.update_ids(np.arange(n, dtype=np.uint32), st0, inc0, now_ms=1)
    sp = torch.cuda.current_stream().cuda_stream
    for r in range(3):
        ids, us, ui = S.c3_updates(n, 1 << 19, seed=700 + r, base_inc=inc0 + 3 * r)
        d = [torch.from_numpy(ids.view(np.int32)).cuda(), torch.from_numpy(us).cuda(), torch.from_numpy(ui).cuda()]
        app_a = torch.full((len(ids),), 0xEE, dtype=torch.uint8, device="cuda")
        app_b = torch.empty(len(ids), dtype=torch.uint8, device="cuda")
        cut = 24 * 4096
        a.update_range_dev(d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), len(ids), 50 + r, 0, cut,
                           app_a.data_ptr(), stream=sp)
        a.update_range_dev(d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), len(ids), 50 + r, cut, n,
                           app_a.data_ptr(), stream=sp)
        b.update_dev(d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), len(ids), 50 + r, app_b.data_ptr(), stream=sp)
        torch.cuda.synchronize()
        assert torch.equal(app_a, app_b)
        assert a.compute_checksum() == b.checksum
    assert all(np.array_equal(x, y) for x, y in zip(a.dump(), b.dump()))
    with pytest.raises(gpu.RingpopAmdError, match="whole buckets"):
        a.update_range_dev(d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), len(ids), 60, 100, 4096, stream=sp)
    a.close()
    b.close()
