"""Probe: can RCCL run two ranks on one GPU here?  (torchrun --nproc-per-node 2;
both ranks on device 0.)  Prints one line per rank."""
import os
import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
torch.cuda.set_device(0)
try:
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    t = torch.full((4,), float(rank + 1), device="cuda:0")
    dist.all_reduce(t)
    torch.cuda.synchronize()
    print(f"rank {rank}: all_reduce ok {t.tolist()}", flush=True)
    dist.destroy_process_group()
except Exception as exc:
    print(f"rank {rank}: RCCL two-ranks-one-GPU failed: {type(exc).__name__}: {exc}", flush=True)
