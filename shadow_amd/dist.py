"""One process per GPU: PHOLD hosts block-sharded over ranks, one exchange per
conservative round.

Per round:
  1. process   each shard pops its hosts' events before the barrier; new events
               for another shard's hosts are packed per owner rank;
  2. counts    all-to-all of the per-peer counts (G x int64);
  3. events    all-to-all-v of the packed {time, id, dst<<32|src} triples —
               RCCL over xGMI on GPUs (torch.distributed "nccl"), gloo on CPU;
  4. insert    received events go into the destination queues;
  5. window    all-reduce MIN of {next event time, min discovered jump, ~overflow}
               — the window barrier (scheduler.c:386-408, master.c:450-480).

The per-shard compute is a backend: ``EngineShard`` (the HIP engine; product
path) or, in CPU tests only, an oracle-backed shard with the same interface.
Unsigned 64-bit values travel as int64 with the sign bit flipped so that a
signed MIN reduction orders them as unsigned.
"""
from __future__ import annotations

import contextlib
import os
import time

import numpy as np
import torch
import torch.distributed as dist

SIGN = 1 << 63


def u64_to_i64(x: int) -> int:
    return (x ^ SIGN) - (1 << 64) if (x ^ SIGN) >= (1 << 63) else (x ^ SIGN)


def i64_to_u64(x: int) -> int:
    return (x & ((1 << 64) - 1)) ^ SIGN


def owner_bounds(n_hosts: int, world: int):
    return [(g * n_hosts) // world for g in range(world + 1)]


class EngineShard:
    """Product backend: the HIP round engine on this rank's GPU."""

    def __init__(self, cfg, rank, world, device, exchange_cap=None, queue_cap=0):
        from .engine import Engine
        self.dev = torch.device("cuda", device)
        torch.cuda.set_device(self.dev)
        # a dedicated stream: engine kernels, torch ops and the collectives of a
        # round are all ordered on it (torch's default stream has handle 0,
        # which the C-ABI reads as "make your own stream")
        self.stream = torch.cuda.Stream(device=self.dev)
        stream = self.stream.cuda_stream
        n_local = owner_bounds(cfg["n_hosts"], world)[rank + 1] - owner_bounds(cfg["n_hosts"], world)[rank]
        if exchange_cap is None:
            # the boot round stages load events per host: size for it
            exchange_cap = max(4096, n_local * cfg["load"])
        self.cap = exchange_cap
        self.world = world
        self.eng_args = (rank, world)
        self.eng = Engine(cfg, device=device, shard_index=rank, shard_count=world,
                          queue_cap=queue_cap, exchange_cap=exchange_cap, stream=stream)
        self.send = torch.empty((world, exchange_cap, 3), dtype=torch.int64, device=self.dev)
        self.send_counts = torch.zeros(world, dtype=torch.int64, device=self.dev)
        self.red = torch.zeros(3, dtype=torch.int64, device=self.dev)
        self.recv = torch.empty((0, 3), dtype=torch.int64, device=self.dev)

    def stream_ctx(self):
        return torch.cuda.stream(self.stream)

    def boot(self):
        self.eng.boot()

    def process(self):
        self.eng.step_process(self.send.data_ptr(), self.send_counts.data_ptr())
        return self.send, self.send_counts

    def insert(self, recv, n):
        self.recv = recv  # keep alive until the kernel consumed it
        self.eng.step_insert(recv.data_ptr() if n else 0, n)

    def reduce(self):
        self.eng.step_reduce(self.red.data_ptr())
        return self.red

    def window(self, red):
        self.eng.step_window(red.data_ptr())

    def done(self) -> bool:
        return bool(self.eng.stats()["done"])

    def stats(self):
        return self.eng.stats()

    def sync(self):
        self.stream.synchronize()


def _flip(t: torch.Tensor) -> torch.Tensor:
    # unsigned order -> signed order (and back): xor the sign bit
    return torch.bitwise_xor(t, torch.tensor(-(1 << 63), dtype=torch.int64, device=t.device))


def exchange(send: torch.Tensor, send_counts: torch.Tensor, world: int):
    """All-to-all-v of packed triples.  Returns (recv [n, 3], n)."""
    recv_counts = torch.empty_like(send_counts)
    dist.all_to_all_single(recv_counts, send_counts)
    sc = send_counts.tolist()  # host sync on the counts (v1 protocol)
    rc = recv_counts.tolist()
    parts = [send[p, :sc[p]] for p in range(world)]
    flat = torch.cat(parts, 0).reshape(-1) if sum(sc) else send.new_zeros(0)
    recv = send.new_empty(sum(rc) * 3)
    dist.all_to_all_single(recv, flat, [c * 3 for c in rc], [c * 3 for c in sc])
    return recv.reshape(-1, 3), sum(rc)


def run_round(shard, world: int):
    send, counts = shard.process()
    recv, n = exchange(send, counts, world)
    shard.insert(recv, n)
    red = shard.reduce()
    red = _flip(red)
    dist.all_reduce(red, op=dist.ReduceOp.MIN)
    red = _flip(red)
    shard.window(red)


def run(shard, world: int, max_rounds: int = 1 << 62, check_every: int = 16) -> int:
    ctx = shard.stream_ctx() if hasattr(shard, "stream_ctx") else contextlib.nullcontext()
    r = 0
    with ctx:
        while r < max_rounds:
            run_round(shard, world)
            r += 1
            if r % check_every == 0 and shard.done():
                break
    return r


# ------------------------------------------------------------------ bench ----
def _env_rank():
    return int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")), \
        int(os.environ.get("LOCAL_RANK", "0"))


def bench(args):
    """bench.py --gpus N under torch.distributed.run: strong scaling of the 1M-host
    PHOLD over N GPUs.  Returns the JSON dict on rank 0, None elsewhere."""
    from . import phold
    rank, world, local = _env_rank()
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch with "
                         "torch.distributed.run --nproc-per-node N")
    torch.cuda.set_device(local)
    dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    cfg = phold.c4_config(n_hosts=args.hosts)
    shard = EngineShard(cfg, rank, world, local)
    shard.boot()
    run(shard, world, args.warmup, check_every=1 << 30)
    shard.sync()
    s0 = shard.stats()
    dist.barrier()
    shard.sync()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(shard, world, args.steps, check_every=1 << 30)
    shard.sync()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    dist.barrier()
    s1 = shard.stats()
    shard.sync()
    t = torch.tensor([dt], dtype=torch.float64, device=shard.dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    pops = torch.tensor([s1["pops"] - s0["pops"], s1["rounds"] - s0["rounds"], s1["overflow"]],
                        dtype=torch.int64, device=shard.dev)
    dist.all_reduce(pops, op=dist.ReduceOp.SUM)
    tmax = float(t.item())
    total, rounds_sum, ovf = (int(x) for x in pops.tolist())
    dist.destroy_process_group()
    if ovf:
        raise SystemExit(f"exchange/queue overflow during bench ({ovf:#x})")
    if rank != 0:
        return None
    return {
        "metric": "committed events/sec (whole node), 1M-host PHOLD at 1/2/4/8 MI355X; bit-exact",
        "value": total / tmax,
        "unit": "events/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": tmax * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic",
        "config": {"workload": f"PHOLD configs[3]: {args.hosts} hosts x 16, V=1024 log-normal "
                               "latency (median 30 ms, sigma 0.9, min 1 ms), runahead 1 ms, "
                               "weights rule, seed 1",
                   "n_hosts": args.hosts, "events_timed": total,
                   "parallelism": f"hosts block-sharded {world} ways, RCCL all-to-all per round"},
    }
