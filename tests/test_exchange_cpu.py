"""CPU (gloo, world_size 2) test of the sharded simulator's message exchange
(ringpop-node_amd MessageExchange): per-peer counts, then one all-to-all-v of the packed outbox
(per destination: 40-byte headers then 24-byte records) into an inbox holding the sources'
segments in rank order. Host buffers stand in for device buffers (copy = memmove)."""
import ctypes
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _segment(rank, g, nm, nr):
    """rank's segment for destination g: nm headers encoding (rank, g, i), nr records (rank, g, j)."""
    parts = [np.full(40, (rank * 16 + g) * 8 + i % 8, dtype=np.uint8) for i in range(nm)]
    parts += [np.full(24, 200 - (rank * 16 + g + j % 4), dtype=np.uint8) for j in range(nr)]
    return np.concatenate(parts) if parts else np.zeros(0, np.uint8)


def _outbox(rank, G, rnd):
    """Synthetic packed outbox of `rank`: for each destination g, rnd-dependent counts."""
    nm = np.array([(rank * 3 + g * 5 + rnd) % 4 for g in range(G)], dtype=np.uint64)
    nr = np.array([(rank * 7 + g * 2 + rnd) % 6 for g in range(G)], dtype=np.uint64)
    segs = [_segment(rank, g, int(nm[g]), int(nr[g])) for g in range(G)]
    return nm, nr, segs


def _worker(rank, W, port, q, sub=None):
    """W world ranks; with `sub` (a list of world ranks) the exchange runs on that subgroup only,
    with its per-peer counts on a side gloo group (the nccl path's count group, built with local
    synchronization: the ranks outside `sub` never construct anything)."""
    import torch.distributed as dist
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from conftest import load_pkg
    rpa = load_pkg()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    env0 = os.environ.get("GLOO_SOCKET_IFNAME")
    dist.init_process_group("gloo", rank=rank, world_size=W)
    group = None
    if sub is not None:
        group = dist.new_group(ranks=sub, backend="gloo", use_local_synchronization=True) if rank in sub else None
        if rank not in sub:
            q.put((rank, True))
            dist.destroy_process_group()
            return
    x = rpa.MessageExchange(group=group, copy=lambda dst, src, nb: ctypes.memmove(dst, src, nb),
                            side_counts=sub is not None)
    G = x.G
    rank = x.rank
    ok = os.environ.get("GLOO_SOCKET_IFNAME") == env0  # the environment is restored
    if sub is not None:
        ok &= x._cgroup is not None and x._cgroup is not group
    for rnd in range(3):
        nm, nr, segs = _outbox(rank, G, rnd)
        out = np.concatenate(segs + [np.zeros(1, np.uint8)])
        box = {}

        def alloc(in_nm, in_nr):
            box["b"] = np.zeros(max(1, int(in_nm.sum()) * 40 + int(in_nr.sum()) * 24), np.uint8)
            return box["b"].ctypes.data

        in_nm, in_nr = x.exchange(nm, nr, out.ctypes.data, alloc)
        # expected: sources in rank order, each source's segment for this rank
        want, want_nm, want_nr = [], [], []
        for s in range(G):
            snm, snr, ssegs = _outbox(s, G, rnd)
            want.append(ssegs[rank])
            want_nm.append(int(snm[rank]))
            want_nr.append(int(snr[rank]))
        ok &= in_nm.tolist() == want_nm and in_nr.tolist() == want_nr
        w = np.concatenate(want)
        ok &= np.array_equal(box["b"][:w.size], w)
    q.put((sub[rank] if sub is not None else rank, bool(ok)))
    dist.destroy_process_group()


def test_message_exchange_gloo_two_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert res == {0: True, 1: True}


def test_message_exchange_on_a_subgroup_with_side_counts():
    """the exchange built on a subgroup (world 3, ranks {0, 2}) with its counts on a
    side gloo group; rank 1 takes no part in either group's creation."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, 3, port, q, [0, 2])) for r in range(3)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert res == {0: True, 1: True, 2: True}


@pytest.mark.parametrize("capacity,world", [(1, 1), (4096, 2), (4 * 4096 + 1234, 2), (4 * 4096 + 1234, 3),
                                            (1 << 22, 8), (100_000, 8), (5, 4)])
def test_part_membership_partition_covers_ids(rpa, capacity, world):
    """PartMembership's id runs (host logic, no device): whole 4,096-id buckets, in rank order,
    disjoint, covering every id of the table, the last one open-ended; what
    rp_members_update_range_dev requires of a range."""
    B = rpa.PartMembership.BUCKET
    runs = [rpa.PartMembership.partition(capacity, world, r) for r in range(world)]
    assert runs[0][1] == 0 and runs[-1][2] >= capacity
    for (_, lo, hi), (_, lo2, _) in zip(runs, runs[1:]):
        assert hi == lo2 and lo <= hi
    for _, lo, hi in runs:
        assert lo % B == 0 and hi % B == 0
