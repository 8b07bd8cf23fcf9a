"""GPU parity of the sharded simulator (C5 path): the nodes split over G shard handles with the
four per-round message exchanges must reproduce the unsharded simulator exactly — every node's
checksum after every round, the convergence round, the stats and final views.

- in one process (ShardedGossipSim: rp_sim_exchange_local between shard handles), G = 2, 3, 4
  and uneven partitions;
- across processes (DistGossipSim over torch.distributed, two ranks sharing cuda:0 with the
  gloo backend: the bytes are staged through host memory; with nccl = RCCL on a multi-GPU
  node the same protocol moves them over xGMI)."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from test_sim_gpu import synth

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _case(n, k, seed):
    S = synth()
    return [S.c2_addr(i) for i in range(n)], S.c3_members(n)[2], S.kill_set(n, k, seed)


@pytest.mark.parametrize("n,k,seed,susp,G,bounds", [
    (300, 6, 3, 25, 2, None),
    (500, 5, 3, 25, 3, None),
    (777, 40, 9, 7, 4, None),
    (400, 8, 5, 10, 3, [0, 7, 390, 400]),
])
def test_sharded_matches_unsharded(gpu, n, k, seed, susp, G, bounds):
    names, inc0, dead = _case(n, k, seed)
    ref = gpu.GossipSim(names, inc0, dead, seed=seed, suspicion_rounds=susp)
    sh = gpu.ShardedGossipSim(names, inc0, dead, G, seed=seed, suspicion_rounds=susp,
                              bounds=None if bounds is None else np.array(bounds, dtype=np.uint32))
    conv_r = conv_s = None
    for r in range(55):
        ref.step()
        sh.step()
        assert np.array_equal(ref.checksums(), sh.checksums()), "round %d" % r
        if conv_r is None and ref.converged():
            conv_r = r
        if conv_s is None and sh.converged():
            conv_s = r
    assert conv_r == conv_s is not None
    assert ref.stats() == sh.stats()
    for v in (0, n // 3, n - 1):
        a, b = ref.view(v), sh.view(v)
        assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    sh.close()
    ref.close()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _join_events(n, k, seed):
    """The dist worker's "join" scenario (tests/workers/dist_sim_worker.py)."""
    _, _, dead = _case(n, k, seed)
    live = np.flatnonzero(dead == 0)
    crashed = np.random.default_rng(seed).permutation(live)[:12]
    ev = [(3, "kill", int(v)) for v in sorted(crashed)]
    return ev + [(9, "join", int(v)) for v in sorted(crashed[:6])] + [(9, "join", int(v)) for v in np.flatnonzero(dead)[:2]]


def _run_dist(gpu, tmp_path, G, backend, n=400, k=6, seed=7, susp=25, rounds=45, scenario=None, timeout=100):
    out = str(tmp_path / "dist.npz")
    port = _free_port()
    worker = os.path.join(REPO, "tests", "workers", "dist_sim_worker.py")
    procs = []
    for r in range(G):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK="0", WORLD_SIZE=str(G), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, worker, str(n), str(k), str(seed), str(susp), str(rounds),
                                       out, backend] + ([scenario] if scenario else []), env=env))
    rcs = [p.wait(timeout=timeout) for p in procs]
    assert rcs == [0] * G
    d = np.load(out)
    names, inc0, dead = _case(n, k, seed)
    ref = gpu.GossipSim(names, inc0, dead, seed=seed, suspicion_rounds=susp,
                        events=_join_events(n, k, seed) if scenario == "join" else ())
    conv = -1
    for r in range(rounds):
        ref.step()
        assert np.array_equal(ref.checksums(), d["checksums"][r]), "round %d" % r
        if conv < 0 and ref.converged():
            conv = r
    assert conv == int(d["conv"]) >= 0
    assert [ref.stats()[x] for x in gpu._STAT_NAMES] == d["stats"].tolist()
    assert int(d["xbytes"]) > 0


def test_dist_two_ranks_gloo_matches_unsharded(gpu, tmp_path):
    _run_dist(gpu, tmp_path, 2, "gloo")


def test_dist_one_rank_nccl_matches_unsharded(gpu, tmp_path):
    """The RCCL transport (device tensors, rp_copy on torch's stream, all_to_all_single over
    nccl) on the one GPU of the box; a multi-GPU node runs the same code with G ranks."""
    _run_dist(gpu, tmp_path, 1, "nccl")


def test_dist_two_ranks_gloo_joins_match_unsharded(gpu, tmp_path):
    """Join events across ranks: the join exchange buffer is summed over torch.distributed."""
    _run_dist(gpu, tmp_path, 2, "gloo", scenario="join")


def test_dist_four_ranks_gloo_joins_match_unsharded(gpu, tmp_path):
    """The 8-GPU run's shape across processes at a smaller scale: 4 ranks (sharing the box's GPU,
    gloo transport), n = 2000 with crashes at round 3 and joins at round 9 (rp_sim_join_export /
    import across all four shards), checked round by round against the unsharded simulator."""
    _run_dist(gpu, tmp_path, 4, "gloo", n=2000, k=20, rounds=50, scenario="join", timeout=200)
