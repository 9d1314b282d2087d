"""ctypes binding of libshadowgpu.so (include/shadowgpu.h).

The library is built in-tree by shadow_amd/build.py.  There is no fallback: a
missing library raises, and engine creation fails loudly without a gfx950 GPU.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_PKG = os.path.dirname(os.path.abspath(__file__))
# SG_LIB (A/B experiments only): another in-tree build of the same library,
# e.g. shadow_amd/libshadowgpu_v.so from `python -m shadow_amd.build --variant v -DX=1`
LIB_PATH = os.path.join(_PKG, os.environ.get("SG_LIB", "libshadowgpu.so"))

SG_OK, SG_ERR_INVAL, SG_ERR_NOMEM, SG_ERR_HIP, SG_ERR_OVERFLOW, SG_ERR_STATE, SG_ERR_NODEV = range(7)
SG_ATTACH_MODULO, SG_ATTACH_RANDOM = 0, 1
SG_DST_UNIFORM_FLOOR, SG_DST_WEIGHTS = 0, 1
SG_WINDOW_FIXED, SG_WINDOW_DISCOVERED = 0, 1
SG_WORKLOAD_PHOLD, SG_WORKLOAD_GOSSIP = 0, 1
ONE_MS = 1_000_000
SIMTIME_MAX = (1 << 64) - 2
RAND_MAX = 2147483647

u32p = np.ctypeslib.ndpointer(np.uint32, flags="C_CONTIGUOUS")
u64p = np.ctypeslib.ndpointer(np.uint64, flags="C_CONTIGUOUS")
i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
f64p = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")


class SgError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"libshadowgpu error {code}: {msg}")
        self.code = code


class PholdParams(C.Structure):
    _fields_ = [(n, C.c_uint32) for n in
                ("n_hosts", "n_vertices", "load", "dst_rule", "window_rule", "queue_cap",
                 "shard_index", "shard_count")] + \
               [(n, C.c_uint64) for n in
                ("end_time", "bootstrap_end", "fixed_jump", "runahead_min", "trace_capacity",
                 "exchange_cap")] + \
               [("workload", C.c_uint32), ("gossip_msgs", C.c_uint32),
                ("gossip_start", C.c_uint64), ("gossip_interval", C.c_uint64)]

    def set_workload(self, cfg: dict):
        self.workload = cfg.get("workload", SG_WORKLOAD_PHOLD)
        self.gossip_msgs = cfg.get("gossip_msgs", 0)
        self.gossip_start = cfg.get("gossip_start", 0)
        self.gossip_interval = cfg.get("gossip_interval", 0)


class PholdTables(C.Structure):
    _fields_ = [("host_vertex", C.c_void_p), ("host_rng", C.c_void_p), ("delay_ns", C.c_void_p),
                ("keep_max", C.c_void_p), ("jump_ms", C.c_void_p), ("weight_thresh", C.c_void_p)]


class RoundStats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in
                ("rounds", "pops", "boots", "sends", "null_dst", "drop_reliability",
                 "drop_endtime", "bumped", "same_round", "overflow", "window_start",
                 "window_end", "done", "min_jump", "next_min_jump", "jmin_ms", "pending",
                 "trace_len", "exchange_steps", "phase")]

    def as_dict(self):
        return {n: int(getattr(self, n)) for n, _ in self._fields_}


class EngineGeom(C.Structure):
    _fields_ = [("bucket_width", C.c_uint64)] + [(n, C.c_uint32) for n in
                ("ring_buckets", "chunk_events", "chunks", "partition_hosts", "partitions",
                 "partition_cap", "stage_cap")]

    def as_dict(self):
        return {n: int(getattr(self, n)) for n, _ in self._fields_}


KERNEL_CLASSES = ("process", "insert", "plan", "gather", "exchange")  # enum sg_kernel_class


class WindowState(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in ("min_jump", "next_min_jump", "min_jump_config", "end_time")]


class XLinkDesc(C.Structure):
    _fields_ = [(n, C.c_uint32) for n in ("fenced", "fused", "shared_device", "selftest_steps",
                                          "selftest_fused", "pad_")] + \
               [("selftest_bad", C.c_uint64), ("steps", C.c_uint64)]

    def as_dict(self):
        return {n: int(getattr(self, n)) for n, _ in self._fields_ if n != "pad_"}


TRACE_DTYPE = np.dtype([("time", "<u8"), ("seq", "<u8"), ("host", "<u4"), ("src", "<u4"),
                        ("pos", "<u8")])

_lib = None

EXPORTS = [
    "sg_last_error", "sg_abi_version", "sg_rand_r", "sg_random_next_double",
    "sg_random_next_uint", "sg_seed_chain", "sg_attach_hosts", "sg_keep_threshold",
    "sg_build_paths", "sg_build_weight_thresholds", "sg_window_note_latency", "sg_window_next",
    "sg_topology_lognormal", "sg_graphml_load", "sg_graph_free", "sg_graph_info", "sg_graph_vertex",
    "sg_graph_edge", "sg_graph_attach", "sg_graph_paths", "sg_build_path_tables", "sg_engine_create", "sg_engine_destroy", "sg_engine_boot",
    "sg_engine_run", "sg_engine_enqueue_round", "sg_engine_sync", "sg_engine_stats",
    "sg_engine_host_state", "sg_engine_host_range", "sg_engine_active_hosts", "sg_engine_event_moves", "sg_engine_gather_paths", "sg_engine_debug_inject", "sg_engine_trace", "sg_engine_windows",
    "sg_engine_stream", "sg_engine_exchange_rows", "sg_engine_set_exchange_cap",
    "sg_engine_exchange_peak", "sg_engine_step_send", "sg_engine_step_recv",
    "sg_engine_enqueue_rounds", "sg_comm_unique_id", "sg_comm_create", "sg_comm_destroy",
    "sg_engine_run_steps", "sg_engine_set_graph", "sg_engine_graph_prepare", "sg_engine_kernel_times",
    "sg_engine_set_timing", "sg_engine_set_timing_mask", "sg_comm_available", "sg_engine_path_counters", "sg_engine_path_counts", "sg_engine_barrier_timers", "sg_engine_barrier_times", "sg_engine_geometry", "sg_engine_stamps", "sg_policy_create", "sg_policy_destroy", "sg_policy_add_host",
    "sg_policy_thread_hosts", "sg_policy_push", "sg_policy_pop", "sg_policy_next_time",
    "sg_policy_remaining", "sg_policy_ops_gpu", "sg_policy_ops_gpu_error", "sg_policy_ops_gpu_policy",
    "sg_policy_kernel_profile", "sg_policy_kernel_stats", "sg_sched_run_phold",
    "sg_sched_run_phold_paths", "sg_path_cache_create", "sg_path_cache_destroy", "sg_path_cache_lookup",
    "sg_path_cache_stats", "sg_xlink_create", "sg_xlink_handle", "sg_xlink_attach", "sg_xlink_selftest",
    "sg_xlink_status", "sg_xlink_info", "sg_xlink_debug_withhold", "sg_xlink_destroy",
    "sg_engine_run_steps_xlink",
]


def lib():
    """Load libshadowgpu.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} is missing: build it with `python -m shadow_amd.build` "
                           "(there is no CPU fallback)")
    L = C.CDLL(LIB_PATH)
    L.sg_last_error.restype = C.c_char_p
    L.sg_rand_r.argtypes = [C.POINTER(C.c_uint32)]
    L.sg_rand_r.restype = C.c_int32
    L.sg_random_next_double.argtypes = [C.POINTER(C.c_uint32)]
    L.sg_random_next_double.restype = C.c_double
    L.sg_random_next_uint.argtypes = [C.POINTER(C.c_uint32)]
    L.sg_random_next_uint.restype = C.c_uint32
    L.sg_seed_chain.argtypes = [C.c_uint32, C.c_uint32, C.POINTER(C.c_uint32),
                                C.POINTER(C.c_uint32), u32p]
    L.sg_attach_hosts.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32, u32p, u32p, u32p]
    L.sg_keep_threshold.argtypes = [C.c_double]
    L.sg_keep_threshold.restype = C.c_int32
    L.sg_build_paths.argtypes = [C.c_uint32, f64p, f64p, C.c_void_p, u64p, i32p, u32p]
    L.sg_build_weight_thresholds.argtypes = [C.c_uint32, f64p, i32p]
    L.sg_window_note_latency.argtypes = [C.POINTER(WindowState), C.c_double]
    L.sg_window_note_latency.restype = None
    L.sg_window_next.argtypes = [C.POINTER(WindowState), C.c_uint64, C.POINTER(C.c_uint64),
                                 C.POINTER(C.c_uint64)]
    L.sg_topology_lognormal.argtypes = [C.c_uint32, C.c_uint64, C.c_double, C.c_double,
                                        C.c_double, C.c_double, f64p, f64p]
    L.sg_engine_create.argtypes = [C.POINTER(PholdParams), C.POINTER(PholdTables), C.c_int,
                                   C.c_void_p, C.POINTER(C.c_void_p)]
    for f in ("sg_engine_destroy", "sg_engine_boot", "sg_engine_enqueue_round", "sg_engine_sync"):
        getattr(L, f).argtypes = [C.c_void_p]
    L.sg_engine_run.argtypes = [C.c_void_p, C.c_uint64, C.c_uint32]
    L.sg_engine_stats.argtypes = [C.c_void_p, C.POINTER(RoundStats)]
    L.sg_engine_host_state.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    L.sg_engine_host_range.argtypes = [C.c_void_p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
    L.sg_engine_active_hosts.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
    L.sg_engine_event_moves.argtypes = [C.c_void_p] + [C.POINTER(C.c_uint64)] * 3
    L.sg_engine_gather_paths.argtypes = [C.c_void_p] + [C.POINTER(C.c_uint64)] * 2
    L.sg_engine_debug_inject.argtypes = [C.c_void_p]
    L.sg_engine_trace.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.POINTER(C.c_uint64)]
    L.sg_engine_windows.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.POINTER(C.c_uint64)]
    L.sg_engine_stream.argtypes = [C.c_void_p]
    L.sg_engine_stream.restype = C.c_void_p
    L.sg_engine_exchange_rows.argtypes = [C.c_void_p, C.POINTER(C.c_uint64)]
    L.sg_engine_set_exchange_cap.argtypes = [C.c_void_p, C.c_uint64]
    L.sg_engine_exchange_peak.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.c_int]
    L.sg_engine_step_send.argtypes = [C.c_void_p, C.c_void_p]
    L.sg_engine_step_recv.argtypes = [C.c_void_p, C.c_void_p]
    L.sg_engine_kernel_times.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_uint64)]
    L.sg_engine_set_timing.argtypes = [C.c_void_p, C.c_int]
    L.sg_engine_set_timing_mask.argtypes = [C.c_void_p, C.c_uint32]
    L.sg_comm_available.argtypes = []
    L.sg_engine_geometry.argtypes = [C.c_void_p, C.POINTER(EngineGeom)]
    L.sg_engine_stamps.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.POINTER(C.c_uint64)]
    L.sg_engine_path_counters.argtypes = [C.c_void_p, C.c_int]
    L.sg_engine_barrier_timers.argtypes = [C.c_void_p, C.c_int]
    L.sg_engine_barrier_times.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.POINTER(C.c_uint64)]
    L.sg_engine_path_counts.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.POINTER(C.c_uint64)]
    L.sg_engine_enqueue_rounds.argtypes = [C.c_void_p, C.c_uint64]
    L.sg_comm_unique_id.argtypes = [C.c_void_p]
    L.sg_comm_create.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_void_p)]
    L.sg_comm_destroy.argtypes = [C.c_void_p]
    L.sg_engine_run_steps.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64]
    L.sg_engine_set_graph.argtypes = [C.c_void_p, C.c_uint32]
    L.sg_engine_graph_prepare.argtypes = [C.c_void_p]
    L.sg_xlink_create.argtypes = [C.c_void_p, C.POINTER(C.c_void_p)]
    L.sg_xlink_handle.argtypes = [C.c_void_p, C.c_void_p]
    L.sg_xlink_attach.argtypes = [C.c_void_p, C.c_void_p]
    L.sg_xlink_selftest.argtypes = [C.c_void_p, C.c_uint32, C.POINTER(C.c_uint64)]
    L.sg_xlink_status.argtypes = [C.c_void_p, C.POINTER(C.c_uint32)]
    L.sg_xlink_info.argtypes = [C.c_void_p, C.POINTER(XLinkDesc)]
    L.sg_xlink_debug_withhold.argtypes = [C.c_void_p, C.c_uint64, C.c_uint32]
    L.sg_xlink_destroy.argtypes = [C.c_void_p]
    L.sg_engine_run_steps_xlink.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64]
    _lib = L
    return L


def check(rc: int):
    if rc != SG_OK:
        raise SgError(rc, lib().sg_last_error().decode(errors="replace"))
