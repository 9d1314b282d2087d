"""TEST INFRASTRUCTURE — ctypes binding of the CPU oracle (oracle/liborc.so).

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg
may import this module; the product path (``shadow_amd``) never does.  The
oracle restates the reference's scheduling semantics on the CPU (see orc.c for
the file:line citations and DESIGN.md §Oracle for how it is pinned).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liborc.so")
_lib = None

u32p = np.ctypeslib.ndpointer(np.uint32, flags="C_CONTIGUOUS")
u64p = np.ctypeslib.ndpointer(np.uint64, flags="C_CONTIGUOUS")
i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
f64p = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")

MODE_HOST, MODE_SERIAL = 0, 1


class OrcParams(C.Structure):
    _fields_ = [(n, C.c_uint32) for n in
                ("n_hosts", "n_vertices", "load", "dst_rule", "window_rule", "mode",
                 "first_host", "n_local")] + \
               [(n, C.c_uint64) for n in
                ("end_time", "bootstrap_end", "fixed_jump", "runahead_min", "trace_capacity")] + \
               [("workload", C.c_uint32), ("gossip_msgs", C.c_uint32),
                ("gossip_start", C.c_uint64), ("gossip_interval", C.c_uint64)]


class OrcStats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in
                ("rounds", "pops", "boots", "sends", "null_dst", "drop_reliability",
                 "drop_endtime", "bumped", "same_round", "pending", "window_start",
                 "window_end", "done", "min_jump", "next_min_jump", "jmin_ms", "trace_len")]

    def as_dict(self):
        return {n: int(getattr(self, n)) for n, _ in self._fields_}


EVENT_DTYPE = np.dtype([("time", "<u8"), ("seq", "<u8"), ("dst", "<u4"), ("src", "<u4"),
                        ("msg", "<u4"), ("pad", "<u4")])
TRACE_DTYPE = np.dtype([("time", "<u8"), ("seq", "<u8"), ("host", "<u4"), ("src", "<u4"),
                        ("pos", "<u8")])


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        L.orc_create.restype = C.c_void_p
        L.orc_create.argtypes = [C.POINTER(OrcParams), u32p, u32p, u64p, i32p, u32p, C.c_void_p]
        L.orc_destroy.argtypes = [C.c_void_p]
        L.orc_error.restype = C.c_char_p
        for f in ("orc_boot", "orc_run_serial", "orc_round_process"):
            getattr(L, f).argtypes = [C.c_void_p]
            getattr(L, f).restype = C.c_int
        L.orc_run.argtypes = [C.c_void_p, C.c_uint64]
        L.orc_run.restype = C.c_int64
        L.orc_outbox.argtypes = [C.c_void_p, C.POINTER(C.c_void_p)]
        L.orc_outbox.restype = C.c_size_t
        L.orc_outbox_clear.argtypes = [C.c_void_p]
        L.orc_ingest.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
        L.orc_ingest.restype = C.c_int
        L.orc_local_min.argtypes = [C.c_void_p]
        L.orc_local_min.restype = C.c_uint64
        L.orc_local_jmin.argtypes = [C.c_void_p]
        L.orc_local_jmin.restype = C.c_uint64
        L.orc_window_apply.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64]
        L.orc_window_apply.restype = C.c_int
        L.orc_stats_get.argtypes = [C.c_void_p, C.POINTER(OrcStats)]
        L.orc_host_state.argtypes = [C.c_void_p, u64p, u64p, u32p, u64p]
        L.orc_trace.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
        L.orc_trace.restype = C.c_size_t
        L.orc_windows.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
        L.orc_windows.restype = C.c_size_t
        L.orc_path_counts.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
        L.orc_path_counts.restype = C.c_size_t
        L.orc_set_ordered_discovery.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int,
                                                C.c_int]
        L.orc_probe_hash.argtypes = [C.c_void_p, C.POINTER(C.c_uint64)]
        L.orc_probe_hash.restype = C.c_uint64
        L.orc_digest_mix.argtypes = [C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint64]
        L.orc_digest_mix.restype = C.c_uint64
        L.orc_rand.argtypes = [C.POINTER(C.c_uint32)]
        L.orc_rand.restype = C.c_int32
        L.orc_seed_chain.argtypes = [C.c_uint32, C.c_uint32, C.POINTER(C.c_uint32),
                                     C.POINTER(C.c_uint32), u32p]
        L.orc_attach.argtypes = [C.c_uint32, C.c_uint32, C.c_int, u32p, u32p, u32p]
        L.orc_build_paths.argtypes = [C.c_uint32, f64p, f64p, C.c_void_p, u64p, i32p, u32p]
        L.orc_weight_thresholds.argtypes = [C.c_uint32, f64p, i32p]
        _lib = L
    return _lib


# ---------------------------------------------------------------- setup -----
def rand_r_stream(seed: int, n: int) -> np.ndarray:
    st = C.c_uint32(seed)
    return np.array([lib().orc_rand(C.byref(st)) for _ in range(n)], dtype=np.int64)


def seed_chain(seed: int, n: int):
    node = np.zeros(max(n, 1), np.uint32)
    a, b = C.c_uint32(), C.c_uint32()
    lib().orc_seed_chain(seed, n, C.byref(a), C.byref(b), node)
    return a.value, b.value, node[:n]


def attach(node_seeds: np.ndarray, n_vertices: int, rule: int):
    n = len(node_seeds)
    v = np.zeros(n, np.uint32)
    r = np.zeros(n, np.uint32)
    lib().orc_attach(n, n_vertices, rule, np.ascontiguousarray(node_seeds, np.uint32), v, r)
    return v, r


def build_paths(latency_ms, edge_loss, vertex_loss=None):
    lat = np.ascontiguousarray(latency_ms, np.float64)
    V = int(round(np.sqrt(lat.size)))
    el = np.ascontiguousarray(edge_loss, np.float64)
    d = np.zeros(V * V, np.uint64)
    k = np.zeros(V * V, np.int32)
    j = np.zeros(V * V, np.uint32)
    vl = None if vertex_loss is None else np.ascontiguousarray(vertex_loss, np.float64)
    lib().orc_build_paths(V, lat.ravel(), el.ravel(),
                          None if vl is None else vl.ctypes.data, d, k, j)
    return d, k, j


def weight_thresholds(weights):
    w = np.ascontiguousarray(weights, np.float64)
    out = np.zeros(len(w), np.int32)
    lib().orc_weight_thresholds(len(w), w, out)
    return out


# ------------------------------------------------------------ simulation ----
class Sim:
    """One oracle instance (a whole simulation, or one shard of it)."""

    def __init__(self, cfg, mode=MODE_HOST, first_host=0, n_local=None, trace_capacity=0):
        """cfg: a dict with the PHOLD parameters and tables (see
        tests/phold_cases.py); the tables come from the oracle's own setup
        restatements so the product's host code is checked, not reused."""
        L = lib()
        p = OrcParams()
        p.n_hosts = cfg["n_hosts"]
        p.n_vertices = cfg["n_vertices"]
        p.load = cfg["load"]
        p.dst_rule = cfg["dst_rule"]
        p.window_rule = cfg["window_rule"]
        p.mode = mode
        p.first_host = first_host
        p.n_local = cfg["n_hosts"] if n_local is None else n_local
        p.end_time = cfg["end_time"]
        p.bootstrap_end = cfg.get("bootstrap_end", 0)
        p.fixed_jump = cfg.get("fixed_jump", 0)
        p.runahead_min = cfg.get("runahead_min", 0)
        p.trace_capacity = trace_capacity
        p.workload = cfg.get("workload", 0)
        p.gossip_msgs = cfg.get("gossip_msgs", 0)
        p.gossip_start = cfg.get("gossip_start", 0)
        p.gossip_interval = cfg.get("gossip_interval", 0)
        self.p = p
        self._keep = [np.ascontiguousarray(cfg[k]) for k in
                      ("host_vertex", "host_rng", "delay_ns", "keep_max", "jump_ms")]
        wt = cfg.get("weight_thresh")
        self._wt = None if wt is None else np.ascontiguousarray(wt, np.int32)
        self.h = L.orc_create(C.byref(p), *self._keep,
                              None if self._wt is None else self._wt.ctypes.data)
        if not self.h:
            raise RuntimeError(L.orc_error().decode())
        self._destroy = L.orc_destroy  # held so interpreter shutdown can still free
        if cfg.get("discovery") == "ordered":  # the reference's path cache in this oracle's pop order
            pc = cfg["paths"]
            self._pc = [np.ascontiguousarray(pc["latency_ms"], np.float64),
                        np.ascontiguousarray(pc["kind"], np.uint8),
                        np.ascontiguousarray(pc["attached"], np.uint8)]
            if mode != MODE_HOST or (n_local is not None and n_local != cfg["n_hosts"]):
                raise ValueError("ordered discovery needs the whole simulation in host order (MODE_HOST)")
            if L.orc_set_ordered_discovery(self.h, *[a.ctypes.data for a in self._pc], int(pc["complete"]),
                                           int(pc["directed"])):
                raise RuntimeError(L.orc_error().decode())

    def close(self):
        if getattr(self, "h", None):
            self._destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def boot(self):
        assert lib().orc_boot(self.h) == 0

    def run(self, max_rounds=1 << 62):
        r = lib().orc_run(self.h, max_rounds)
        if r < 0:
            raise RuntimeError(lib().orc_error().decode())
        return r

    def run_serial(self):
        assert lib().orc_run_serial(self.h) == 0

    def round_process(self):
        assert lib().orc_round_process(self.h) == 0

    def outbox(self) -> np.ndarray:
        ptr = C.c_void_p()
        n = lib().orc_outbox(self.h, C.byref(ptr))
        if n == 0:
            return np.zeros(0, EVENT_DTYPE)
        buf = (C.c_char * (n * EVENT_DTYPE.itemsize)).from_address(ptr.value)
        out = np.frombuffer(buf, EVENT_DTYPE).copy()
        lib().orc_outbox_clear(self.h)
        return out

    def ingest(self, ev: np.ndarray):
        ev = np.ascontiguousarray(ev, EVENT_DTYPE)
        assert lib().orc_ingest(self.h, ev.ctypes.data, len(ev)) == 0

    def local_min(self) -> int:
        return lib().orc_local_min(self.h)

    def local_jmin(self) -> int:
        return lib().orc_local_jmin(self.h)

    def window_apply(self, gmin: int, gjmin: int) -> bool:
        return bool(lib().orc_window_apply(self.h, gmin, gjmin))

    def stats(self) -> dict:
        s = OrcStats()
        lib().orc_stats_get(self.h, C.byref(s))
        return s.as_dict()

    def host_state(self):
        n = self.p.n_local
        d, p, e = (np.zeros(n, np.uint64) for _ in range(3))
        r = np.zeros(n, np.uint32)
        lib().orc_host_state(self.h, d, p, r, e)
        return {"digest": d, "pops": p, "rng": r, "ev": e}

    def trace(self) -> np.ndarray:
        n = lib().orc_trace(self.h, None, 0)
        out = np.zeros(n, TRACE_DTYPE)
        lib().orc_trace(self.h, out.ctypes.data, n)
        return out

    def windows(self) -> np.ndarray:
        n = lib().orc_windows(self.h, None, 0)
        out = np.zeros(2 * n, np.uint64)
        lib().orc_windows(self.h, out.ctypes.data, n)
        return out.reshape(n, 2)

    def path_counts(self) -> np.ndarray:
        n = lib().orc_path_counts(self.h, None, 0)
        out = np.zeros(n, np.uint64)
        lib().orc_path_counts(self.h, out.ctypes.data, n)
        return out

    def probe_hash(self):
        m = C.c_uint64()
        h = lib().orc_probe_hash(self.h, C.byref(m))
        return h, m.value


def digest_mix(pos, time, src, seq) -> int:
    return lib().orc_digest_mix(pos, time, src, seq)


# --------------------------------------------------- CPU policies (baseline) --
_hsglib = None
HSGLIB_PATH = os.path.join(_HERE, "libhsglib.so")


def faithful_available() -> bool:
    """libhsglib.so (host_steal.c with priority_queue.c's GLib heap) is built."""
    if not os.path.exists(HSGLIB_PATH):
        try:
            build()
        except Exception:  # noqa: BLE001 — no GLib on this machine
            return False
    return os.path.exists(HSGLIB_PATH)


def cpu_policy_ops(steal: bool, n_threads: int, n_hosts: int, faithful: bool = False):
    """host_steal / host_single restatements (oracle/host_steal.c) as a
    shadow_amd.policy.PolicyOps vtable, for the Shadow-style round driver.
    faithful: the per-host queue is priority_queue.c's heap with its GLib
    hash-table position map (libhsglib.so); otherwise plain binary heaps."""
    global _hsglib
    from shadow_amd.policy import PolicyOps
    if faithful:
        if not faithful_available():
            raise RuntimeError("oracle/libhsglib.so is not built (GLib headers absent)")
        if _hsglib is None:
            _hsglib = C.CDLL(HSGLIB_PATH)
        L = _hsglib
    else:
        L = lib()
    L.orc_policy_ops_cpu.argtypes = [C.c_int, C.c_uint32, C.c_uint32, C.POINTER(PolicyOps)]
    ops = PolicyOps()
    if L.orc_policy_ops_cpu(int(steal), n_threads, n_hosts, C.byref(ops)) != 0:
        raise RuntimeError("orc_policy_ops_cpu failed")
    ops._owner = "cpu"
    ops._lib = L  # keeps the library that holds the vtable loaded
    return ops
