"""Probe: can two RCCL ranks share one GPU (a 1-GPU box rehearsal of a real multi-rank collective)?
torchrun --nproc-per-node 2 scripts/dev/rccl_two_ranks_one_gpu.py"""
import os

import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
x = torch.full((1024,), float(rank + 1), device="cuda:0")
dist.all_reduce(x)
torch.cuda.synchronize()
print(f"rank {rank}: all_reduce -> {x[0].item()} (expected 3.0)", flush=True)
dist.destroy_process_group()
