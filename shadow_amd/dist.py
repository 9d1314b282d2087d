"""One process per GPU: PHOLD hosts block-sharded over ranks, ONE collective
per step and no host synchronisation inside the round loop.

A step:
  1. step_send   a process step pops each shard's hosts' events before the
                 barrier; new events for another shard's hosts go to a per-peer
                 outbox.  Every step copies up to exchange_cap outbox events
                 per peer into a fixed-size block behind a header that carries
                 the shard's MIN next time, its min discovered latency and its
                 overflow flags;
  2. all-to-all  one all_to_all_single of equal [rows, 2] int64 blocks —
                 RCCL over xGMI on GPUs (torch.distributed "nccl"), gloo on CPU;
  3. step_recv   local + received events into the destination queues, then the
                 window from the G headers: the MIN "all-reduce" of the window
                 barrier (scheduler.c:386-408, master.c:450-480) rides on the
                 all-to-all.  If a sender still has outbox leftovers every shard
                 turns the next step into a drain step (same window, exchange
                 only); the decision is taken on the device, identically on
                 every shard, so the host never waits on a count.

The per-shard compute is a backend: ``EngineShard`` (the HIP engine; product
path) or, in CPU tests only, an oracle-backed shard with the same interface.
Unsigned 64-bit values travel as int64 bit patterns.
"""
from __future__ import annotations

import contextlib
import os
import time

import torch
import torch.distributed as dist

def owner_bounds(n_hosts: int, world: int):
    return [(g * n_hosts) // world for g in range(world + 1)]


def default_exchange_cap(n_local: int, world: int) -> int:
    """Per-peer rows per step before tuning: a shard's hosts emit well under one
    event per host per round in steady state, about 1/world of them per peer."""
    c = max(4096, -(-n_local // (2 * world)))
    return -(-c // 256) * 256


class EngineShard:
    """Product backend: the HIP round engine on this rank's GPU."""

    def __init__(self, cfg, rank, world, device, exchange_cap=None, queue_cap=0, stream=None,
                 trace_capacity=0):
        from .engine import Engine
        self.dev = torch.device("cuda", device)
        torch.cuda.set_device(self.dev)
        # a dedicated stream: engine kernels, torch ops and the collective of a
        # step are all ordered on it (torch's default stream has handle 0,
        # which the C-ABI reads as "make your own stream")
        self.stream = stream if stream is not None else torch.cuda.Stream(device=self.dev)
        b = owner_bounds(cfg["n_hosts"], world)
        n_local = b[rank + 1] - b[rank]
        if exchange_cap is None:
            exchange_cap = default_exchange_cap(n_local, world)
        self.world = world
        self.rank = rank
        self.comm = None  # the native step loop's communicator (enable_native)
        self.xl = None    # the xGMI peer exchange (enable_xlink), preferred to comm once set
        self.eng = Engine(cfg, device=device, shard_index=rank, shard_count=world,
                          queue_cap=queue_cap, exchange_cap=exchange_cap,
                          trace_capacity=trace_capacity, stream=self.stream.cuda_stream)
        self._alloc()

    row_words = 2  # int64 words per exchange row (include/shadowgpu.h, step_send)

    def _alloc(self):
        rows = self.eng.exchange_rows()
        self.rows = rows
        self.send = torch.zeros((self.world, rows, self.row_words), dtype=torch.int64, device=self.dev)
        self.recv = torch.zeros_like(self.send)

    def _all_ok(self, ok: bool) -> bool:
        """Every rank's flag, AND-reduced over the default group."""
        t = torch.tensor([1 if ok else 0], dtype=torch.int64)
        if _backend() == "nccl":
            t = t.to(self.dev)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return bool(int(t.item()))

    def enable_native(self, graph_batch: int = 0):
        """Issue whole steps from C (sg_engine_run_steps) over a communicator of
        libshadowgpu's own, made from a unique id rank 0 broadcasts over the
        default process group; graph_batch > 0 replays captured hipGraphs.

        Every decision is collective, so all ranks take the native loop or none:
        each rank's local checks (RCCL opens and exports its symbols, the device
        index is valid) come first with no collective, the flags are
        AND-reduced, rank 0's id is broadcast with its own flag, and after the
        collective ncclCommInitRank a second AND-reduce confirms every rank got a
        communicator (a rank that did not releases nothing, the others close
        theirs).  Raises on every rank when the native loop is unavailable.
        A rank whose ncclCommInitRank itself fails after the others entered it
        can still leave them blocked inside RCCL's init: that failure is
        RCCL's, after every check this side can make locally."""
        from .engine import Comm
        local_ok = Comm.available() and 0 <= self.dev.index < torch.cuda.device_count()
        if not self._all_ok(local_ok):
            raise RuntimeError("RCCL cannot be opened on every rank")
        uid = torch.zeros(129, dtype=torch.uint8)  # [0]: rank 0 made an id; [1:]: the id
        if self.rank == 0:
            try:
                uid[1:].copy_(torch.frombuffer(bytearray(Comm.unique_id()), dtype=torch.uint8))
                uid[0] = 1
            except Exception:  # every rank learns it from the broadcast
                pass
        if _backend() == "nccl":
            u = uid.to(self.dev)
            dist.broadcast(u, 0)
            uid = u.cpu()
        else:
            dist.broadcast(uid, 0)
        if not int(uid[0]):
            raise RuntimeError("rank 0 could not create an RCCL unique id")
        uid = uid[1:]
        comm, err = None, None
        try:
            comm = Comm(bytes(uid.tolist()), self.rank, self.world, self.dev.index)
        except Exception as exc:  # noqa: BLE001 — reported after the agreement below
            err = exc
        if not self._all_ok(comm is not None):
            if comm is not None:
                comm.close()
            raise RuntimeError(f"RCCL communicator creation failed on some rank ({err})")
        self.comm = comm
        self.eng.set_graph(graph_batch)

    def enable_xlink(self, selftest_steps: int = 64):
        """Exchange blocks by xGMI peer stores (sg_xlink) from now on: each rank
        exports its receive region, the 128-byte handles are all-gathered,
        every rank maps its peers', and `selftest_steps` pattern exchanges are
        checked on every rank before the first real step — through the path the
        steps take (the fused push: many workgroups storing into the peers'
        regions, each releasing and taking a ticket, the last one writing the
        headers and arriving).  Collective like enable_native: all ranks take
        the link or none (RuntimeError on every rank otherwise).  Call it once
        exchange_cap is final."""
        from .engine import XLink
        xl, err, h = None, None, bytes(XLink.HANDLE_BYTES)
        try:
            xl = XLink(self.eng)
            h = xl.handle()
        except Exception as exc:  # noqa: BLE001 — every rank learns it below
            err = exc
        if not self._all_ok(xl is not None and err is None):
            self._drop_link(xl)
            raise RuntimeError(f"xGMI exchange region unavailable on some rank ({err})")
        t = torch.frombuffer(bytearray(h), dtype=torch.uint8)
        if _backend() == "nccl":
            t = t.to(self.dev)
        parts = [torch.zeros_like(t) for _ in range(self.world)]
        dist.all_gather(parts, t)
        handles = b"".join(bytes(p.cpu().tolist()) for p in parts)
        try:
            xl.attach(handles)
        except Exception as exc:  # noqa: BLE001
            err = exc
        if not self._all_ok(err is None):
            self._drop_link(xl)
            raise RuntimeError(f"mapping the peers' exchange regions failed on some rank ({err})")
        try:
            bad = xl.selftest(selftest_steps)
        except Exception as exc:  # noqa: BLE001
            bad, err = -1, exc
        if not self._all_ok(bad == 0):
            self._drop_link(xl)
            raise RuntimeError(f"xGMI exchange self-test failed on some rank (this rank: "
                               f"{bad if bad < 0 else hex(bad)}{'' if err is None else ', ' + str(err)})")
        self.xl = xl
        self.xl_info = xl.info()

    def _drop_link(self, xl):
        dist.barrier()  # no peer still stores into this rank's region
        if xl is not None:
            xl.close()

    def close_native(self):
        """Drop the exchange link (after every rank stopped stepping), the
        captured graphs, then the communicator (RCCL frees captured
        collectives' resources with their graph)."""
        if getattr(self, "xl", None) is not None:
            xl, self.xl = self.xl, None
            try:
                xl.check()
            finally:
                self._drop_link(xl)
        if getattr(self, "comm", None) is not None:
            self.eng.set_graph(0)
            self.sync()
            self.comm.close()
            self.comm = None

    @property
    def native(self) -> bool:
        return self.xl is not None or self.comm is not None

    def run_native(self, n: int, check: bool = True):
        """n native steps; over the xGMI link, check=True then synchronises and
        raises if a wait timed out (naming the senders that never arrived)."""
        if self.xl is not None:
            self.eng.run_steps_xlink(self.xl, n)
            if check:
                self.xl.check()
        else:
            self.eng.run_steps(self.comm, self.send.data_ptr(), self.recv.data_ptr(), n)

    def check_link(self):
        """Raises if a wait of the xGMI link timed out (no-op without one)."""
        if getattr(self, "xl", None) is not None:
            self.xl.check()

    def stream_ctx(self):
        return torch.cuda.stream(self.stream)

    def boot(self):
        self.eng.boot()

    def pre(self) -> torch.Tensor:
        self.eng.step_send(self.send.data_ptr())
        return self.send

    def post(self):
        self.eng.step_recv(self.recv.data_ptr())

    def set_exchange_cap(self, cap: int):
        """Between steps; every rank must pass the same value."""
        self.sync()
        self.eng.set_exchange_cap(cap)
        self._alloc()

    def exchange_peak(self, reset: bool = False) -> int:
        return self.eng.exchange_peak(reset)

    def done(self) -> bool:
        return bool(self.eng.stats()["done"])

    def fingerprint(self) -> int:
        """This shard's term of the host-state fingerprint (sums to the unsharded one)."""
        from .trace import state_fingerprint
        hs = self.eng.host_state()
        return state_fingerprint(self.eng.first_host, hs["digest"], hs["pops"], hs["rng"], hs["ev"])

    def stats(self):
        return self.eng.stats()

    def sync(self):
        self.stream.synchronize()


def _all_to_all(recv: torch.Tensor, send: torch.Tensor):
    if send.is_cuda and _backend() == "gloo":
        # rehearsal only (several ranks on one GPU, where RCCL refuses to run):
        # gloo exchanges host tensors
        r = torch.empty(send.shape, dtype=send.dtype)
        dist.all_to_all_single(r, send.cpu())
        recv.copy_(r)
    else:
        dist.all_to_all_single(recv, send)


_BACKEND = None


def _backend():
    """The default group's backend, looked up once (the step loop is host-bound
    on small shards: every microsecond of Python per step shows)."""
    global _BACKEND
    if _BACKEND is None:
        _BACKEND = dist.get_backend()
    return _BACKEND


def run_step(shard, world: int):
    send = shard.pre()
    _all_to_all(shard.recv, send)
    shard.post()


def run(shard, world: int, max_steps: int = 1 << 62, check_every: int = 16, check_link: bool = True) -> int:
    """Run steps until the simulation is done (checked every check_every steps)
    or max_steps; returns the steps run.  check_link=False leaves the xGMI
    link's time-out check to the caller (the bench's timed region: the check
    synchronises)."""
    if getattr(shard, "native", False):
        n = 0
        while n < max_steps:
            k = min(check_every - n % check_every, max_steps - n)
            shard.run_native(k, check=check_link)
            n += k
            if n % check_every == 0 and shard.done():
                break
        return n
    ctx = shard.stream_ctx() if hasattr(shard, "stream_ctx") else contextlib.nullcontext()
    n = 0
    with ctx:
        while n < max_steps:
            run_step(shard, world)
            n += 1
            if n % check_every == 0 and shard.done():
                break
    return n


def _any_rank(flag: bool, dev) -> bool:
    t = torch.tensor([1 if flag else 0], dtype=torch.int64)
    if _backend() == "nccl":
        t = t.to(dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return bool(int(t.item()))


def run_until_round(shard, world: int, rounds: int, check_every: int = 8) -> int:
    """Run steps until every shard has completed `rounds` windows (or is done),
    in batches of check_every steps (so it may run past `rounds`).  The decision
    is collective: every rank runs the same number of steps."""
    n = 0
    dev = getattr(shard, "dev", None)
    while True:
        st = shard.stats()
        if not _any_rank(not (st["done"] or st["rounds"] >= rounds), dev):
            return n
        n += run(shard, world, check_every, check_every=1 << 30)


def finish_round(shard, world: int, max_steps: int = 1 << 16) -> dict:
    """Run single steps until every rank is at a round boundary (phase 0) or
    done; returns this shard's stats there."""
    dev = getattr(shard, "dev", None)
    for _ in range(max_steps):
        st = shard.stats()
        if not _any_rank(not (st["phase"] == 0 or st["done"]), dev):
            return st
        run(shard, world, 1, check_every=1 << 30)
    raise RuntimeError("no round boundary within max_steps drain steps")


# ------------------------------------------------------------------ bench ----
def _env_rank():
    return int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")), \
        int(os.environ.get("LOCAL_RANK", "0"))


def _gather_rows(vals, dev):
    """All ranks' float rows, to every rank (list of lists)."""
    t = torch.tensor(vals, dtype=torch.float64, device=dev)
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [o.tolist() for o in out]


def _cuda_sync():
    if torch.cuda.is_available():
        torch.cuda.synchronize()


def bench(args, make_shard=None):
    """bench.py --gpus N under torch.distributed.run: the workload (args.cfg,
    bench.py --workload; configs[3]'s 1M-host PHOLD by default) over N GPUs
    (strong scaling: the host count stays fixed).  Returns the JSON dict on
    rank 0, None elsewhere.  make_shard(cfg, rank, world, device) builds the
    rank's shard: EngineShard (the product) unless a CPU test passes its own."""
    from . import phold
    from . import workloads as WL
    from ._lib import KERNEL_CLASSES
    rank, world, local = _env_rank()
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch with "
                         "torch.distributed.run --nproc-per-node N")
    dev = 0 if args.same_device else local
    if make_shard is None:
        make_shard = EngineShard
        torch.cuda.set_device(dev)
    if args.dist_backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
    else:  # rehearsal of the multi-rank path on one GPU (or a CPU test)
        dist.init_process_group(args.dist_backend)
    # small collectives live where the backend wants them
    cdev = torch.device("cuda", dev) if args.dist_backend == "nccl" else torch.device("cpu")
    wname = getattr(args, "workload", "c4")
    wl = WL.get(wname)
    # the config is built here, once torch has set up the device: ranks that
    # loaded the native library before it saw no HIP device
    cfg = getattr(args, "cfg", None)
    if cfg is None:
        cfg = wl["build"](args.hosts) if hasattr(args, "workload") else phold.c4_config(n_hosts=args.hosts)
        args.cfg = cfg
    args.hosts = cfg["n_hosts"]
    shard = make_shard(cfg, rank, world, dev)
    if args.dist_backend == "nccl" and not args.py_steps:
        try:
            shard.enable_native(args.graph)
        except Exception as exc:  # the same on every rank (enable_native decides collectively)
            import sys
            print(f"native step loop unavailable ({exc}); driving steps from Python",
                  file=sys.stderr, flush=True)
            shard.comm = None
    native = shard.comm is not None
    shard.boot()
    # warmup: the boot round (its outbox drains over several steps), then size
    # the exchange blocks from the steady-state per-peer peak, the same on every rank
    run_until_round(shard, world, 2)
    shard.exchange_peak(reset=True)
    run_until_round(shard, world, 2 + max(args.warmup, 8))
    peak = torch.tensor([shard.exchange_peak()], dtype=torch.int64, device=cdev)
    dist.all_reduce(peak, op=dist.ReduceOp.MAX)
    cap = -(-(int(peak.item()) * 5 // 4 + 256) // 256) * 256
    shard.set_exchange_cap(cap)
    exch = "RCCL all-to-all" if native else f"{args.dist_backend} all-to-all"
    want = getattr(args, "exchange", "rccl")
    xinfo = {"requested": want}
    if want in ("auto", "xgmi") and hasattr(shard, "enable_xlink"):
        try:
            shard.enable_xlink()
            exch = "xGMI peer stores (sg_xlink)"
            xinfo.update(shard.xl_info, taken=True)
        except Exception as exc:  # the same on every rank (enable_xlink decides collectively)
            if want == "xgmi":
                raise
            import sys
            print(f"xGMI exchange unavailable ({exc}); keeping the {exch}", file=sys.stderr, flush=True)
            xinfo.update(taken=False, reason=str(exc)[:300])
    run(shard, world, 8, check_every=1 << 30)
    shard.sync()
    s0 = shard.stats()
    dist.barrier()
    shard.sync()
    _cuda_sync()
    t0 = time.perf_counter()
    run(shard, world, args.steps, check_every=1 << 30, check_link=False)
    shard.sync()
    _cuda_sync()
    dt = time.perf_counter() - t0
    if hasattr(shard, "check_link"):
        shard.check_link()  # a timed-out exchange wait raises here, naming the sender
    dist.barrier()
    s1 = shard.stats()
    t = torch.tensor([dt], dtype=torch.float64, device=cdev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    # the parity point: a step boundary where the round is complete on every
    # rank.  A drain step (phase 1) has popped the next window's events before
    # `rounds` counts it, so finish it first (untimed; the drain decision is the
    # same on every rank, the check is collective all the same)
    end = finish_round(shard, world)
    fp = shard.fingerprint()  # this shard's term of the end-of-region state fingerprint
    tot = torch.tensor([s1["pops"] - s0["pops"], s1["rounds"] - s0["rounds"],
                        s1["exchange_steps"] - s0["exchange_steps"], end["overflow"],
                        int(s1["done"]), fp - (1 << 64 if fp >= 1 << 63 else 0)],
                       dtype=torch.int64, device=cdev)
    dist.all_reduce(tot, op=dist.ReduceOp.SUM)
    tmax = float(t.item())
    total, rounds_sum, steps_sum, ovf, done_sum, fp = (int(x) for x in tot.tolist())
    fp &= (1 << 64) - 1
    end_round = end["rounds"]
    # per-rank kernel times over the next steps (HIP events on the engine stream;
    # the exchange class is this rank's RCCL all-to-all: its wait for the slowest
    # rank plus the transfer, the barrier idle time of scheduler.c:380-389), with
    # the algorithmic bytes the same steps moved: each rank's roofline per kernel
    kr = max(1, min(args.steps, args.kernel_rounds))
    eng = getattr(shard, "eng", None)
    if eng is not None:
        from .roofline import proc_bytes, scatter_bytes
        sa, a1, mv1 = shard.stats(), eng.active_hosts()[0], eng.event_moves()
        eng.set_timing(True)
        run(shard, world, kr, check_every=1 << 30)
        kt = eng.kernel_times()
        eng.set_timing(False)
        sb, a2, mv2 = shard.stats(), eng.active_hosts()[0], eng.event_moves()
        moves = {k: mv2[k] - mv1[k] for k in mv2}
        vals = [kt[c][0] * 1e3 / kr for c in KERNEL_CLASSES]  # us per step per class
        vals += [kt["process"][1], proc_bytes(sb["pops"] - sa["pops"], a2 - a1),
                 kt["insert"][1], scatter_bytes(moves), kt["exchange"][1],
                 float(world * shard.rows * shard.row_words * 8)]  # exchange bytes this rank sends per step
        rows = _gather_rows(vals, cdev)
    else:
        rows = None
    shard.close_native()
    dist.destroy_process_group()
    global _BACKEND
    _BACKEND = None
    if ovf:
        raise SystemExit(f"queue/outbox overflow during bench ({ovf:#x})")
    if rounds_sum == 0 or done_sum:
        raise SystemExit(f"simulation ended early: {rounds_sum // world} rounds timed, done on "
                         f"{done_sum} of {world} ranks")
    if rank != 0:
        return None
    res = {
        "metric": wl["metric"](cfg),
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
        "config": {"workload": wl["describe"](cfg), "name": wname,
                   "n_hosts": cfg["n_hosts"], "events_timed": total,
                   "rounds_timed": rounds_sum // world, "drain_steps": (steps_sum - rounds_sum) // world,
                   "exchange_cap": cap,
                   "parallelism": f"hosts block-sharded {world} ways, one exchange per step: {exch}",
                   "exchange": exch,
                   "xlink": xinfo,
                   "step_loop": "native (sg_engine_run_steps_xlink)" if exch.startswith("xGMI") else
                                f"native (sg_engine_run_steps, hipGraph batch {args.graph})" if native
                                else "python"},
        # bench.py checks these against the oracle fixture and drops them
        "_end_round": end_round, "_fingerprint": fp,
    }
    if rows is not None:
        nk = len(KERNEL_CLASSES)
        res["per_rank_us_per_step"] = {
            "classes": list(KERNEL_CLASSES), "steps": kr, "rows": [r[:nk] for r in rows],
            "note": "HIP events around every launch on each rank's engine stream (they inflate "
                    "each kernel by a few us); 'exchange' is the step's block exchange (xGMI push "
                    "+ arrival wait, or the RCCL all-to-all): wait for the slowest rank + transfer "
                    "(barrier idle, scheduler.c:380-389); the Python step loop (--py-steps, gloo) "
                    "leaves it untimed"}
        res["roofline"] = dist_roofline(rows, nk, kr, KERNEL_CLASSES)
    return res


def dist_roofline(rows, nk, steps, classes):
    """The N > 1 line's roofline: per rank, k_proc and k_scatter's algorithmic
    bytes per launch over their average launch time (HIP events) against 8 TB/s,
    and the exchange's µs and bytes per step; the top-level fields are the
    slowest rank's k_proc (the dominant kernel)."""
    from .roofline import HBM_PEAK_GBS, kernel_line
    per_rank = []
    for r in rows:
        us = dict(zip(classes, r[:nk]))
        pn, pb, sn, sb, xn, xb = r[nk:nk + 6]
        kp = kernel_line(pb / max(pn, 1), us["process"] * 1e-6 * steps / max(pn, 1))
        ks = kernel_line(sb / max(sn, 1), us["insert"] * 1e-6 * steps / max(sn, 1))
        per_rank.append({"k_proc": kp, "k_scatter": ks,
                         "exchange": {"avg_us": us["exchange"] * steps / xn if xn else None,
                                      "bytes_per_step": xb, "timed": bool(xn)}})
    slow = max(range(len(per_rank)), key=lambda i: per_rank[i]["k_proc"]["avg_us"])
    kp = per_rank[slow]["k_proc"]
    return {"bound": "hbm", "kernel": "k_proc", "rank": slow, "achieved": kp["achieved"],
            "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": kp["frac"], "traffic": None,
            "avg_launch_us": kp["avg_us"], "alg_bytes_per_launch": kp["alg_bytes_per_launch"],
            "timing_rounds": steps, "per_rank": per_rank,
            "per_kernel": {k: {"frac_min": min(p[k]["frac"] for p in per_rank),
                               "frac_max": max(p[k]["frac"] for p in per_rank),
                               "avg_us_max": max(p[k]["avg_us"] for p in per_rank)}
                           for k in ("k_proc", "k_scatter")},
            "timing_method": "HIP events as each launch's dispatch-packet timestamps, steps after "
                             "the timed region; traffic (PMC) is profiled at N = 1 only"}
