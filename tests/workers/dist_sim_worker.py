"""One rank of a DistGossipSim run (launched by tests/test_sim_shard_gpu.py as WORLD_SIZE
processes on the same box). Rank 0 writes every round's gathered checksums, the convergence
round and the stats to OUT (npz).

    RANK=r WORLD_SIZE=g MASTER_ADDR=127.0.0.1 MASTER_PORT=p python dist_sim_worker.py n k seed susp rounds out backend [join]
"""
import importlib.util
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def main():
    n, k, seed, susp, rounds = (int(x) for x in sys.argv[1:6])
    out, backend = sys.argv[6], sys.argv[7]
    rpa = load("ringpop_node_amd", os.path.join(REPO, "ringpop-node_amd", "__init__.py"))
    S = load("rp_synth", os.path.join(REPO, "ringpop-node_amd", "synth.py"))
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        dist.init_process_group("gloo")
    names = [S.c2_addr(i) for i in range(n)]
    inc0 = S.c3_members(n)[2]
    dead = S.kill_set(n, k, seed)
    events = ()
    if len(sys.argv) > 8 and sys.argv[8] == "join":  # kills at round 3, some rejoin at 9 (+ 2 never-up nodes)
        live = np.flatnonzero(dead == 0)
        crashed = np.random.default_rng(seed).permutation(live)[:12]
        events = [(3, "kill", int(v)) for v in sorted(crashed)]
        events += [(9, "join", int(v)) for v in sorted(crashed[:6])] + [(9, "join", int(v)) for v in np.flatnonzero(dead)[:2]]
    sim = rpa.DistGossipSim(names, inc0, dead, seed=seed, suspicion_rounds=susp, device=local, events=events)
    cks, conv = [], -1
    for r in range(rounds):
        sim.step()
        cks.append(sim.checksums())
        if conv < 0 and sim.converged():
            conv = r
    st = sim.stats()
    if dist.get_rank() == 0:
        np.savez(out, checksums=np.stack(cks), conv=conv, stats=np.array([st[x] for x in rpa._STAT_NAMES]),
                 xbytes=sim.exchange_bytes)
    sim.close()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
