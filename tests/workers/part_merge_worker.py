"""One rank of a PartMembership run (launched by tests/test_merge_shard_gpu.py as WORLD_SIZE
processes on the same box): the member table partitioned by id across the ranks; every rank
holds the whole batch stream and folds the changes of its own ids (rp_members_update_range_dev),
and after every batch all ranks bring the rows together and compute the checksum (a
collective). Rank 0 writes the per-batch checksums, the per-batch applied flags (each change's
flag from the rank owning its id) and the final table to OUT (npz).

    RANK=r WORLD_SIZE=g MASTER_ADDR=127.0.0.1 MASTER_PORT=p python part_merge_worker.py n k nbatch out backend
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


def batches(S, n, k, nbatch, inc0):
    """The initial table, fresh C3 batches, a repeated batch (applies nothing), and one address
    with 300 changes in a batch (past the bucket fold's LDS list: the overflow fold)."""
    out = [(np.arange(n, dtype=np.uint32), np.zeros(n, np.uint8), inc0)]
    for b in range(nbatch):
        out.append(S.c3_updates(n, k, seed=60 + b, base_inc=inc0 + 3 * b))
        if b == 1:
            out.append(out[-1])
    ids, us, ui = S.c3_updates(n, k, seed=98, base_inc=inc0 + 3 * nbatch)
    hot = n - 7  # on the last rank's ids
    ids = np.concatenate([ids, np.full(300, 5, np.uint32), np.full(300, hot, np.uint32)])
    us = np.concatenate([us, np.arange(300, dtype=np.uint8) % 4, np.arange(300, dtype=np.uint8) % 3])
    ui = np.concatenate([ui, inc0[5] + 3 * nbatch + np.arange(300, dtype=np.int64) % 5,
                         inc0[hot] + 3 * nbatch + np.arange(300, dtype=np.int64) % 4])
    out.append((ids, us, ui))
    return out


def main():
    n, k, nbatch = (int(x) for x in sys.argv[1:4])
    out, backend = sys.argv[4], sys.argv[5]
    rpa = load("ringpop_node_amd", os.path.join(REPO, "ringpop-node_amd", "__init__.py"))
    S = load("rp_synth", os.path.join(REPO, "ringpop-node_amd", "synth.py"))
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    names, _, inc0 = S.c3_members(n)
    m = rpa.PartMembership(whoami=names[0], capacity=n, device=local)
    assert m.intern(names) == list(range(n))
    stream = torch.cuda.current_stream()
    cks, apps = [], []
    for b, (ids, us, ui) in enumerate(batches(S, n, k, nbatch, inc0)):
        kk = len(ids)
        d = [torch.from_numpy(np.ascontiguousarray(ids).view(np.int32)).cuda(), torch.from_numpy(us).cuda(),
             torch.from_numpy(ui).cuda()]
        app = torch.full((kk,), 0xEE, dtype=torch.uint8, device="cuda")
        m.update_dev(d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), kk, 1434500000000 + b, app.data_ptr(),
                     stream=stream.cuda_stream)
        torch.cuda.synchronize()
        a = app.cpu().numpy()
        own = (ids >= m.id_lo) & (ids < m.id_hi)
        assert np.all(a[~own] == 0xEE), "a change of another rank's ids was written"
        parts = [torch.zeros(kk, dtype=torch.uint8) for _ in range(world)]
        dist.all_gather(parts, torch.from_numpy(np.where(own, a, 0).astype(np.uint8)))
        apps.append(np.sum([p.numpy().astype(np.int64) for p in parts], axis=0).astype(np.uint8))
        cks.append(m.compute_checksum())
    ex, st, inc = m.dump()
    if rank == 0:
        np.savez(out, checksums=np.array(cks, dtype=np.int64), ex=ex, st=st, inc=inc,
                 applied=np.concatenate(apps), ranges=np.array([m.id_lo, m.per_ids], dtype=np.int64))
    m.close()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
