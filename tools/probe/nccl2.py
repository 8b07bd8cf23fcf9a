"""Probe: two nccl (RCCL) ranks on the one GPU of a box (is a world-2 RCCL run possible here?).
    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 tools/probe/nccl2.py"""
import os
import torch
import torch.distributed as dist

dist.init_process_group("nccl")
r = dist.get_rank()
torch.cuda.set_device(0)
t = torch.ones(4, device="cuda") * (r + 1)
dist.all_reduce(t)
print("rank", r, "all_reduce", t.tolist(), flush=True)
dist.destroy_process_group()
