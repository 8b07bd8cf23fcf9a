"""bench.py's launch contract on the GPU box: `python bench.py --gpus 2` (no torchrun) starts two
rank processes itself, the C5-path simulator is sharded over them (DistGossipSim: message
exchange by all-to-all-v; gloo here because both ranks share the box's one GPU — the driver's
8-GPU node runs the same code over RCCL), and rank 0 prints ONE JSON line reporting n_gpus = 2
with every rank's keys counted."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(gpus, extra, env_extra=None):
    env = dict(os.environ, **(env_extra or {}))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(gpus)] + extra,
                       env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


SMALL = ["--steps", "2", "--warmup", "1", "--batch-log2", "18", "--no-merge", "--no-wire", "--no-cpu",
         "--sim-n", "0", "--sim5-n", "3000"]


def test_bench_two_ranks_spawned(gpu):
    out = _bench(2, SMALL, {"RP_BENCH_BACKEND": "gloo"})
    assert out["n_gpus"] == 2
    assert out["config"]["total_keys"] == 2 * 2 * (1 << 18)
    assert out["sim_c5"]["n_gpus"] == 2 and out["sim_c5"]["converged"]
    assert out["sim_c5"]["exchange_bytes_per_round_rank0"] > 0
    for k in ("metric", "value", "unit", "roofline", "ms_per_step", "scaling"):
        assert k in out


def test_bench_one_gpu_schema(gpu):
    out = _bench(1, SMALL)
    assert out["n_gpus"] == 1 and out["roofline"]["frac"] > 0
    assert out["sim_c5"]["round_ms"]["max"] >= out["sim_c5"]["round_ms"]["p50"]
    assert out["sim_c5"]["traffic"]["records"] > 0


def test_bench_four_ranks_spawned_with_merge(gpu):
    """`bench.py --gpus 4`: four ranks (gloo; they share the box's GPU), the C5-path simulator
    sharded four ways, the C3 merge as four replicas with batch-strided checksums
    (DistMembership) and the fold partitioned by member id (PartMembership); rank 0 reports
    n_gpus = 4 for each."""
    small = [x for x in SMALL if x != "--no-merge"] + ["--part-log2", "16"]
    out = _bench(4, small, {"RP_BENCH_BACKEND": "gloo"})
    assert out["n_gpus"] == 4
    assert out["config"]["total_keys"] == 4 * 2 * (1 << 18)
    assert out["sim_c5"]["n_gpus"] == 4 and out["sim_c5"]["converged"]
    assert out["merge"]["n_gpus"] == 4 and out["merge"]["updates_per_s"] > 0
    assert isinstance(out["merge"]["checksum"], int)
    # the id-partitioned fold (PartMembership) at 2^16 members / updates, four ways
    fp = out["merge"]["fold_large_partitioned"]
    assert fp["n_gpus"] == 4 and fp["members"] == 1 << 16 and fp["ms_per_batch"] > 0
    # the exchange's host and device time per round, shown with -rP
    print("sim_c5 exchange:", json.dumps({k: v for k, v in out["sim_c5"].items()
                                          if k.startswith("exchange") or k in ("rounds", "round_ms")}))
