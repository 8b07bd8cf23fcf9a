"""One rank of a DistMembership run (launched by tests/test_merge_shard_gpu.py as WORLD_SIZE
processes on the same box): every rank folds the same C3-shaped batch stream on its own replica
of the member table; checksums are divided by batch (b % G == rank). Rank 0 writes the gathered
per-batch checksums and its final table to OUT (npz).

    RANK=r WORLD_SIZE=g MASTER_ADDR=127.0.0.1 MASTER_PORT=p python dist_merge_worker.py n k nbatch out backend [each]

With `each`, every rank reads `m.latest_checksum()` after every batch (a collective)
with a 2-entry device history, so the record is drained by every read; rank 0 also writes those
per-batch reads.
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
    """The test's batch stream: the initial table, fresh C3 batches, a repeated batch (applies
    nothing: the checksum carries over), and a hot address beyond the grouped fold's limit."""
    out = [(np.arange(n, dtype=np.uint32), np.zeros(n, np.uint8), inc0)]
    for b in range(nbatch):
        out.append(S.c3_updates(n, k, seed=40 + b, base_inc=inc0 + 3 * b))
        if b == 2:
            out.append(out[-1])
    ids, us, ui = S.c3_updates(n, k, seed=99, base_inc=inc0 + 3 * nbatch)
    ids = np.concatenate([ids, np.full(40, 5, np.uint32)])
    us = np.concatenate([us, np.arange(40, dtype=np.uint8) % 4])
    ui = np.concatenate([ui, inc0[5] + 3 * nbatch + np.arange(40, dtype=np.int64) % 3])
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
    names, _, inc0 = S.c3_members(n)
    each = len(sys.argv) > 6 and sys.argv[6] == "each"
    m = rpa.DistMembership(whoami=names[0], capacity=n, device=local, history_cap=2 if each else 1 << 16)
    assert m.intern(names) == list(range(n))
    stream = torch.cuda.current_stream()
    keep, reads = [], []
    for b, (ids, us, ui) in enumerate(batches(S, n, k, nbatch, inc0)):
        d = [torch.from_numpy(np.ascontiguousarray(ids).view(np.int32)).cuda(), torch.from_numpy(us).cuda(),
             torch.from_numpy(ui).cuda()]
        keep.append(d)
        m.update_dev(d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), len(ids), 1434500000000 + b,
                     stream=stream.cuda_stream)
        if each:
            reads.append(m.latest_checksum())
    torch.cuda.synchronize()
    try:
        m.checksum
        raise AssertionError("DistMembership.checksum must refuse on G > 1 ranks")
    except rpa.RingpopAmdError:
        pass
    assert m.local_checksum() is not None
    cks = m.checksums()
    ex, st, inc = m.dump()
    if dist.get_rank() == 0:
        np.savez(out, checksums=np.array([-1 if c is None else c for c in cks], dtype=np.int64), ex=ex, st=st,
                 inc=inc, reads=np.array([-1 if c is None else c for c in reads], dtype=np.int64))
    m.close()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
