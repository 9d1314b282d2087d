"""Python handle on the HBM-resident round engine (libshadowgpu, Mode S)."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L


class Engine:
    """One shard of a PHOLD simulation resident on one MI355X.

    Single shard: ``boot(); run(max_rounds)``.  Multi-shard: the distributed
    driver (shadow_amd.dist) calls the step_* methods around its collectives.
    """

    def __init__(self, cfg: dict, *, device: int = 0, shard_index: int = 0, shard_count: int = 1,
                 queue_cap: int = 0, trace_capacity: int = 0, exchange_cap: int = 0,
                 stream: int | None = None):
        lib = L.lib()
        if cfg.get("discovery") == "ordered" and not cfg["paths"]["complete"]:
            raise ValueError("ordered path discovery (the reference's lookup-order cache) runs in the "
                             "CPU-worker driver and the oracle; the engine's jump table is source-wide")
        p = L.PholdParams()
        p.n_hosts = cfg["n_hosts"]
        p.n_vertices = cfg["n_vertices"]
        p.load = cfg["load"]
        p.dst_rule = cfg["dst_rule"]
        p.window_rule = cfg["window_rule"]
        p.queue_cap = queue_cap
        p.shard_index = shard_index
        p.shard_count = shard_count
        p.end_time = cfg["end_time"]
        p.bootstrap_end = cfg.get("bootstrap_end", 0)
        p.fixed_jump = cfg.get("fixed_jump", 0)
        p.runahead_min = cfg.get("runahead_min", 0)
        p.trace_capacity = trace_capacity
        p.exchange_cap = exchange_cap
        p.set_workload(cfg)
        self.params = p
        self._arrays = [np.ascontiguousarray(cfg["host_vertex"], np.uint32),
                        np.ascontiguousarray(cfg["host_rng"], np.uint32),
                        np.ascontiguousarray(cfg["delay_ns"], np.uint64),
                        np.ascontiguousarray(cfg["keep_max"], np.int32),
                        np.ascontiguousarray(cfg["jump_ms"], np.uint32)]
        wt = cfg.get("weight_thresh")
        self._wt = None if wt is None else np.ascontiguousarray(wt, np.int32)
        t = L.PholdTables(*[a.ctypes.data for a in self._arrays],
                          None if self._wt is None else self._wt.ctypes.data)
        h = C.c_void_p()
        L.check(lib.sg_engine_create(C.byref(p), C.byref(t), device, stream, C.byref(h)))
        self.h = h
        lo, n = C.c_uint32(), C.c_uint32()
        L.check(lib.sg_engine_host_range(h, C.byref(lo), C.byref(n)))
        self.first_host, self.n_local = lo.value, n.value

    def close(self):
        if getattr(self, "h", None):
            L.lib().sg_engine_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    # -------------------------------------------------------- single shard
    def boot(self):
        L.check(L.lib().sg_engine_boot(self.h))

    def run(self, max_rounds: int = 1 << 62, batch: int = 32):
        L.check(L.lib().sg_engine_run(self.h, max_rounds, batch))

    def enqueue_round(self):
        L.check(L.lib().sg_engine_enqueue_round(self.h))

    def enqueue_rounds(self, n: int):
        """n rounds, no read-back; at most two batches queued."""
        L.check(L.lib().sg_engine_enqueue_rounds(self.h, n))

    def set_graph(self, batch: int):
        """Capture every `batch` rounds / steps into a hipGraph and replay it (0: off)."""
        L.check(L.lib().sg_engine_set_graph(self.h, batch))

    def prepare_graph(self):
        """Capture one batch of rounds now without running it (graphs on)."""
        L.check(L.lib().sg_engine_graph_prepare(self.h))

    def sync(self):
        L.check(L.lib().sg_engine_sync(self.h))

    @property
    def stream(self) -> int:
        return L.lib().sg_engine_stream(self.h) or 0

    # ------------------------------------------------------------- results
    def stats(self) -> dict:
        s = L.RoundStats()
        L.check(L.lib().sg_engine_stats(self.h, C.byref(s)))
        return s.as_dict()

    def active_hosts(self):
        a, e = C.c_uint64(), C.c_uint64()
        L.check(L.lib().sg_engine_active_hosts(self.h, C.byref(a), C.byref(e)))
        return a.value, e.value

    def event_moves(self) -> dict:
        """Cumulative events staged by k_proc, gathered by k_scatter from the
        calendar into partitions, and received events k_scatter routed into
        partitions (several shards)."""
        v = [C.c_uint64() for _ in range(3)]
        L.check(L.lib().sg_engine_event_moves(self.h, *[C.byref(x) for x in v]))
        return dict(zip(("emitted", "gathered", "received"), (x.value for x in v)))

    def gather_paths(self) -> dict:
        """k_scatter launches whose gather took the due list the k_proc before
        guessed (GSpec) and launches that derived it from the bucket words."""
        v = [C.c_uint64() for _ in range(2)]
        L.check(L.lib().sg_engine_gather_paths(self.h, *[C.byref(x) for x in v]))
        return dict(zip(("guessed", "listed"), (x.value for x in v)))

    def debug_inject(self):
        """Test only: corrupt two staged records before the next round's
        k_scatter (sg_engine_debug_inject); the insert role must flag OV_BUG."""
        L.check(L.lib().sg_engine_debug_inject(self.h))

    def host_state(self) -> dict:
        n = self.n_local
        d, p, e = (np.zeros(n, np.uint64) for _ in range(3))
        r = np.zeros(n, np.uint32)
        L.check(L.lib().sg_engine_host_state(self.h, d.ctypes.data, p.ctypes.data, r.ctypes.data,
                                             e.ctypes.data))
        return {"digest": d, "pops": p, "rng": r, "ev": e}

    def trace(self) -> np.ndarray:
        n = C.c_uint64()
        L.check(L.lib().sg_engine_trace(self.h, None, 0, C.byref(n)))
        out = np.zeros(n.value, L.TRACE_DTYPE)
        if n.value:
            L.check(L.lib().sg_engine_trace(self.h, out.ctypes.data, n.value, C.byref(n)))
        return out

    def windows(self) -> np.ndarray:
        n = C.c_uint64()
        L.check(L.lib().sg_engine_windows(self.h, None, 0, C.byref(n)))
        out = np.zeros(2 * n.value, np.uint64)
        if n.value:
            L.check(L.lib().sg_engine_windows(self.h, out.ctypes.data, n.value, C.byref(n)))
        return out.reshape(-1, 2)

    def path_counters(self, enable: bool = True):
        """Count kept sends per (src vertex, dst vertex) from now on (zeroed)."""
        L.check(L.lib().sg_engine_path_counters(self.h, int(enable)))

    def object_counts(self) -> dict:
        """Event objects created and freed so far (object_counter.c:90-230 for
        the Event type): created = boot events + every event a send or a
        schedule made (staged, same-round or dropped at endTime); freed = every
        executed pop + every endTime drop (scheduler.c:343-346).  The
        difference is the events still queued."""
        a, e = C.c_uint64(), C.c_uint64()
        L.check(L.lib().sg_engine_active_hosts(self.h, C.byref(a), C.byref(e)))
        st = self.stats()
        new = st["boots"] + e.value + st["same_round"] + st["drop_endtime"]
        return {"event_new": new, "event_free": st["pops"] + st["drop_endtime"],
                "event_live": st["pending"]}

    def barrier_timers(self, enable: bool = True):
        """Per-partition busy / barrier-idle time from now on (zeroed);
        scheduler.c:380-389's per-worker wait timers, a partition's k_proc
        workgroup as the worker."""
        L.check(L.lib().sg_engine_barrier_timers(self.h, int(enable)))

    def barrier_times(self) -> dict:
        """{"busy_ns": [P], "idle_ns": [P]} since barrier_timers(True)."""
        n = C.c_uint64()
        L.check(L.lib().sg_engine_barrier_times(self.h, None, None, 0, C.byref(n)))
        b, i = np.zeros(n.value, np.uint64), np.zeros(n.value, np.uint64)
        if n.value:
            L.check(L.lib().sg_engine_barrier_times(self.h, b.ctypes.data, i.ctypes.data, n.value, C.byref(n)))
        return {"busy_ns": b, "idle_ns": i}

    def path_counts(self) -> np.ndarray:
        n = C.c_uint64()
        L.check(L.lib().sg_engine_path_counts(self.h, None, 0, C.byref(n)))
        out = np.zeros(n.value, np.uint64)
        if n.value:
            L.check(L.lib().sg_engine_path_counts(self.h, out.ctypes.data, n.value, C.byref(n)))
        return out

    def set_timing(self, on: bool, classes=None):
        """Per-kernel HIP-event timing: every class, or only `classes` (names of
        _lib.KERNEL_CLASSES) — fewer events inflate the timed kernels less."""
        if classes is None:
            L.check(L.lib().sg_engine_set_timing(self.h, int(on)))
        else:
            mask = sum(1 << L.KERNEL_CLASSES.index(c) for c in classes) if on else 0
            L.check(L.lib().sg_engine_set_timing_mask(self.h, mask))

    def kernel_times(self):
        """{class: (total ms, launches)} since set_timing(True), per sg_kernel_class."""
        k = len(L.KERNEL_CLASSES)
        ms = (C.c_double * k)()
        n = (C.c_uint64 * k)()
        L.check(L.lib().sg_engine_kernel_times(self.h, ms, n))
        return {c: (ms[i], n[i]) for i, c in enumerate(L.KERNEL_CLASSES)}

    def geometry(self) -> dict:
        g = L.EngineGeom()
        L.check(L.lib().sg_engine_geometry(self.h, C.byref(g)))
        return g.as_dict()

    def stamps(self) -> np.ndarray:
        """[2P + G3 + G1 + 3, 32] stamps of the last round (SG_STAMPS=1): P rows of
        k_proc phase stamps, one spare row, then one row per k_scatter workgroup
        {start, setup, events, end, role, n}; or empty."""
        n = C.c_uint64()
        L.check(L.lib().sg_engine_stamps(self.h, None, 0, C.byref(n)))
        out = np.zeros(n.value, np.uint64)
        if n.value:
            L.check(L.lib().sg_engine_stamps(self.h, out.ctypes.data, n.value, C.byref(n)))
        return out.reshape(-1, 32)

    # ---------------------------------------------------------- multi shard
    def exchange_rows(self) -> int:
        r = C.c_uint64()
        L.check(L.lib().sg_engine_exchange_rows(self.h, C.byref(r)))
        return r.value

    def set_exchange_cap(self, cap: int):
        L.check(L.lib().sg_engine_set_exchange_cap(self.h, cap))

    def exchange_peak(self, reset: bool = False) -> int:
        r = C.c_uint64()
        L.check(L.lib().sg_engine_exchange_peak(self.h, C.byref(r), int(reset)))
        return r.value

    def step_send(self, send_ptr: int):
        L.check(L.lib().sg_engine_step_send(self.h, send_ptr))

    def step_recv(self, recv_ptr: int):
        L.check(L.lib().sg_engine_step_recv(self.h, recv_ptr))

    def run_steps(self, comm: "Comm", send_ptr: int, recv_ptr: int, n: int):
        """n whole steps (step_send, RCCL all-to-all, step_recv) issued from C."""
        L.check(L.lib().sg_engine_run_steps(self.h, comm.h, send_ptr, recv_ptr, n))

    def run_steps_xlink(self, xl: "XLink", n: int):
        """n whole steps with the exchange as xGMI peer stores (sg_engine_run_steps_xlink)."""
        L.check(L.lib().sg_engine_run_steps_xlink(self.h, xl.h, n))


class XLink:
    """The xGMI peer exchange of one shard (sg_xlink_*): this shard's region of
    uncached device memory, exported as a 128-byte handle (IPC + device); attach() maps the
    peers' regions (all handles in rank order, all-gathered by the caller).
    Steps then run through Engine.run_steps_xlink: each block is stored
    straight into its peer's region, with no collective."""

    HANDLE_BYTES = 128  # IPC handle + PCI bus id (include/shadowgpu.h)

    def __init__(self, eng: "Engine"):
        h = C.c_void_p()
        L.check(L.lib().sg_xlink_create(eng.h, C.byref(h)))
        self.h = h
        self.eng = eng

    def handle(self) -> bytes:
        buf = (C.c_uint8 * self.HANDLE_BYTES)()
        L.check(L.lib().sg_xlink_handle(self.h, buf))
        return bytes(buf)

    def attach(self, handles: bytes):
        buf = (C.c_uint8 * len(handles)).from_buffer_copy(handles)
        L.check(L.lib().sg_xlink_attach(self.h, buf))

    def selftest(self, n_steps: int) -> int:
        """Mismatched words over n_steps pattern exchanges (+2^63 if a wait
        timed out); every shard calls it with the same n_steps."""
        bad = C.c_uint64()
        L.check(L.lib().sg_xlink_selftest(self.h, n_steps, C.byref(bad)))
        return bad.value

    def timed_out_senders(self) -> list:
        """The shards whose arrival a wait of this link gave up on (synchronises
        the engine stream)."""
        t = C.c_uint32()
        L.check(L.lib().sg_xlink_status(self.h, C.byref(t)))
        return [q for q in range(32) if t.value >> q & 1]

    def timed_out(self) -> bool:
        return bool(self.timed_out_senders())

    def check(self):
        """Raises once a wait has timed out, naming the senders that never
        arrived (after the first time-out every later wait returns at once, so
        the steps enqueued behind it finish quickly and the run stops)."""
        bad = self.timed_out_senders()
        if bad:
            raise RuntimeError(f"xGMI exchange: no arrival from shard(s) {bad} within 5 s "
                               f"(shard {self.eng.params.shard_index} of {self.eng.params.shard_count}); the run stopped")

    def info(self) -> dict:
        d = L.XLinkDesc()
        L.check(L.lib().sg_xlink_info(self.h, C.byref(d)))
        return d.as_dict()

    def debug_withhold(self, step: int, peer: int):
        """Tests only: the fused step `step` steps from now skips its arrival at `peer`."""
        L.check(L.lib().sg_xlink_debug_withhold(self.h, step, peer))

    def close(self):
        if getattr(self, "h", None):
            h, self.h = self.h, None
            L.check(L.lib().sg_xlink_destroy(h))


class Comm:
    """An RCCL communicator owned by libshadowgpu (sg_comm_create): rank 0 makes
    the 128-byte unique id, the caller broadcasts it."""

    @staticmethod
    def available() -> bool:
        """RCCL can be opened in this process (no collective is made)."""
        return L.lib().sg_comm_available() == L.SG_OK

    @staticmethod
    def unique_id() -> bytes:
        buf = (C.c_uint8 * 128)()
        L.check(L.lib().sg_comm_unique_id(buf))
        return bytes(buf)

    def __init__(self, uid: bytes, rank: int, world: int, device: int):
        buf = (C.c_uint8 * 128).from_buffer_copy(uid)
        h = C.c_void_p()
        L.check(L.lib().sg_comm_create(buf, rank, world, device, C.byref(h)))
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            L.lib().sg_comm_destroy(self.h)
            self.h = None


def probe_hash(trace: np.ndarray) -> tuple[int, int]:
    """The survey probe's chained trace hash over message pops (boot pops skipped),
    hosts in index order, each host's pops in pop order."""
    t = np.sort(trace, order=["host", "pos"])
    msg = ~((t["src"] == t["host"]) & (t["seq"] == 0))
    t = t[msg]
    h = 5381
    M = (1 << 64) - 1
    for tm, src, seq, host in zip(t["time"].tolist(), t["src"].tolist(), t["seq"].tolist(),
                                  t["host"].tolist()):
        h = ((h * 1000003) & M) ^ ((tm * 31 + src * 7 + seq + host) & M)
    return h, int(msg.sum())
