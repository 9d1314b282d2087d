"""The `gpu` SchedulerPolicy (Mode P) and the Shadow-style round driver.

``run_phold(cfg, n_workers, ops)`` runs the PHOLD workload with real CPU worker
threads (the reference's scheduler.c / worker.c structure, restated in
sg_sched.c) under a policy vtable: ``gpu_ops()`` gives the drop-in `gpu`
policy whose queues, sort and MIN live on the MI355X.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L


class HEvent(C.Structure):
    _fields_ = [("time", C.c_uint64), ("seq", C.c_uint64), ("src", C.c_uint32), ("dst", C.c_uint32)]


ADD_HOST = C.CFUNCTYPE(None, C.c_void_p, C.c_uint32, C.c_uint64)
GET_HOSTS = C.CFUNCTYPE(C.c_uint32, C.c_void_p, C.c_uint64, C.POINTER(C.c_uint32), C.c_uint32)
PUSH = C.CFUNCTYPE(None, C.c_void_p, C.POINTER(HEvent), C.c_uint32, C.c_uint32, C.c_uint64)
POP = C.CFUNCTYPE(C.POINTER(HEvent), C.c_void_p, C.c_uint64)
NEXT = C.CFUNCTYPE(C.c_uint64, C.c_void_p)
FREE = C.CFUNCTYPE(None, C.c_void_p)


class PolicyOps(C.Structure):
    """sg_sched_policy_ops — mirrors struct _SchedulerPolicy (scheduler_policy.h:40-51)."""
    _fields_ = [("data", C.c_void_p), ("add_host", ADD_HOST), ("get_assigned_hosts", GET_HOSTS),
                ("push", PUSH), ("pop", POP), ("get_next_time", NEXT), ("free", FREE)]


class SchedResult(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in ("rounds", "pops", "sends", "drop_reliability",
                                          "drop_endtime", "bumped")] + \
               [("seconds", C.c_double), ("last_window_start", C.c_uint64),
                ("last_window_end", C.c_uint64), ("mark_round", C.c_uint64),
                ("marked_seconds", C.c_double), ("marked_pops", C.c_uint64),
                ("marked_rounds", C.c_uint64), ("profile", C.c_uint64)] + \
               [(n, C.c_double) for n in ("prof_push_s", "prof_pop_s", "prof_next_s", "prof_exec_s",
                                          "prof_barrier_s")] + \
               [("prof_pushes", C.c_uint64), ("prof_pops", C.c_uint64)]

    def as_dict(self):
        return {n: (float if t is C.c_double else int)(getattr(self, n)) for n, t in self._fields_}


class KernelStat(C.Structure):
    """sg_kernel_stat (include/shadowgpu.h): one device kernel class of the policy."""
    _fields_ = [("name", C.c_char * 16), ("launches", C.c_uint64), ("ms", C.c_double), ("alg_bytes", C.c_double)]


def _bind():
    lib = L.lib()
    if not getattr(lib, "_policy_bound", False):
        lib.sg_policy_ops_gpu.argtypes = [C.c_uint32, C.c_uint32, C.c_int, C.POINTER(PolicyOps)]
        lib.sg_policy_ops_gpu_error.argtypes = [C.POINTER(PolicyOps)]
        lib.sg_sched_run_phold.argtypes = [C.POINTER(L.PholdParams), C.POINTER(L.PholdTables),
                                           C.c_uint32, C.c_uint32, C.POINTER(PolicyOps), C.c_uint64,
                                           C.POINTER(SchedResult), C.c_void_p, C.c_void_p,
                                           C.c_void_p, C.c_void_p]
        lib.sg_sched_run_phold_paths.argtypes = [C.POINTER(L.PholdParams), C.POINTER(L.PholdTables),
                                                 C.c_void_p, C.c_uint32, C.c_uint32, C.POINTER(PolicyOps),
                                                 C.c_uint64, C.POINTER(SchedResult), C.c_void_p, C.c_void_p,
                                                 C.c_void_p, C.c_void_p]
        lib.sg_path_cache_create.argtypes = [C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int,
                                             C.POINTER(C.c_void_p)]
        lib.sg_path_cache_destroy.argtypes = [C.c_void_p]
        lib.sg_path_cache_lookup.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint64),
                                             C.POINTER(C.c_double)]
        lib.sg_path_cache_stats.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        lib.sg_policy_ops_gpu_policy.argtypes = [C.POINTER(PolicyOps)]
        lib.sg_policy_ops_gpu_policy.restype = C.c_void_p
        lib.sg_policy_kernel_profile.argtypes = [C.c_void_p, C.c_int, C.c_uint32]
        lib.sg_policy_kernel_stats.argtypes = [C.c_void_p, C.POINTER(KernelStat), C.c_uint32,
                                               C.POINTER(C.c_uint32)]
        lib._policy_bound = True
    return lib


class PathCache:
    """sg_path_cache: the reference's lazy path cache, looked up in the order
    the driver's workers reach their sends (cfg["discovery"] == "ordered", from
    phold.topology_config)."""

    def __init__(self, cfg: dict):
        lib = _bind()
        pc = cfg["paths"]
        self._keep = [np.ascontiguousarray(pc["latency_ms"], np.float64),
                      np.ascontiguousarray(pc["kind"], np.uint8),
                      np.ascontiguousarray(pc["attached"], np.uint8)]
        h = C.c_void_p()
        L.check(lib.sg_path_cache_create(cfg["n_vertices"], *[a.ctypes.data for a in self._keep],
                                         int(pc["complete"]), int(pc["directed"]), C.byref(h)))
        self.h = h
        self._destroy = lib.sg_path_cache_destroy

    def lookup(self, src_vertex: int, dst_vertex: int):
        """(pair index of the path returned, minimum latency stored so far in ms)."""
        k, m = C.c_uint64(), C.c_double()
        L.check(_bind().sg_path_cache_lookup(self.h, src_vertex, dst_vertex, C.byref(k), C.byref(m)))
        return int(k.value), float(m.value)

    def stats(self):
        r, n = C.c_uint64(), C.c_uint64()
        L.check(_bind().sg_path_cache_stats(self.h, C.byref(r), C.byref(n)))
        return {"runs": int(r.value), "stored": int(n.value)}

    def close(self):
        if getattr(self, "h", None):
            self._destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()


def gpu_ops(n_workers: int, n_hosts: int, device: int = 0) -> PolicyOps:
    ops = PolicyOps()
    L.check(_bind().sg_policy_ops_gpu(n_workers, n_hosts, device, C.byref(ops)))
    ops._owner = "gpu"
    return ops


def kernel_profile(ops: PolicyOps, enable: bool = True, skip_rounds: int = 0):
    """Per-kernel device profile of a gpu vtable's policy (sg_policy_kernel_profile):
    the first skip_rounds extractions are not counted."""
    lib = _bind()
    p = lib.sg_policy_ops_gpu_policy(C.byref(ops))
    if not p:
        raise ValueError("not a gpu policy vtable")
    L.check(lib.sg_policy_kernel_profile(p, int(enable), skip_rounds))


def kernel_stats(ops: PolicyOps) -> dict:
    """{kernel: {launches, ms, alg_bytes}} of a gpu vtable's policy (before its free)."""
    lib = _bind()
    p = lib.sg_policy_ops_gpu_policy(C.byref(ops))
    if not p:
        raise ValueError("not a gpu policy vtable")
    out = (KernelStat * 32)()
    n = C.c_uint32()
    L.check(lib.sg_policy_kernel_stats(p, out, 32, C.byref(n)))
    return {out[i].name.decode(): {"launches": int(out[i].launches), "ms": float(out[i].ms),
                                   "alg_bytes": float(out[i].alg_bytes)} for i in range(min(n.value, 32))}


def phold_args(cfg: dict):
    """(sg_phold_params, sg_phold_tables, arrays kept alive) for the CPU-worker
    driver (sg_sched_run_phold)."""
    p = L.PholdParams()
    p.n_hosts = cfg["n_hosts"]
    p.n_vertices = cfg["n_vertices"]
    p.load = cfg["load"]
    p.dst_rule = cfg["dst_rule"]
    p.window_rule = cfg["window_rule"]
    p.end_time = cfg["end_time"]
    p.bootstrap_end = cfg.get("bootstrap_end", 0)
    p.fixed_jump = cfg.get("fixed_jump", 0)
    p.runahead_min = cfg.get("runahead_min", 0)
    p.set_workload(cfg)
    arrs = [np.ascontiguousarray(cfg["host_vertex"], np.uint32),
            np.ascontiguousarray(cfg["host_rng"], np.uint32),
            np.ascontiguousarray(cfg["delay_ns"], np.uint64),
            np.ascontiguousarray(cfg["keep_max"], np.int32),
            np.ascontiguousarray(cfg["jump_ms"], np.uint32)]
    wt = cfg.get("weight_thresh")
    wt = None if wt is None else np.ascontiguousarray(wt, np.int32)
    t = L.PholdTables(*[a.ctypes.data for a in arrs], None if wt is None else wt.ctypes.data)
    return p, t, (arrs, wt)


def default_scheduler_seed(cfg: dict) -> int:
    from .phold import seed_chain
    return seed_chain(cfg.get("seed", 1), 0)[1]  # slave.c:198


def run_phold(cfg: dict, n_workers: int, ops: PolicyOps, max_rounds: int = 1 << 62,
              scheduler_seed: int | None = None, free_ops: bool = True,
              mark_round: int = 0, profile: bool = False) -> dict:
    """Run PHOLD under `ops` with n_workers CPU workers; returns per-host state
    (digest, pops, rng, ev) and the driver's counters/timing."""
    lib = _bind()
    if scheduler_seed is None:
        scheduler_seed = default_scheduler_seed(cfg)
    p, t, _keep = phold_args(cfg)
    n = cfg["n_hosts"]
    dig, pops, ev = (np.zeros(n, np.uint64) for _ in range(3))
    rng = np.zeros(n, np.uint32)
    res = SchedResult()
    res.mark_round = mark_round
    res.profile = int(profile)
    cache = PathCache(cfg) if cfg.get("discovery") == "ordered" else None
    rc = lib.sg_sched_run_phold_paths(C.byref(p), C.byref(t), cache.h if cache else None, n_workers,
                                      scheduler_seed, C.byref(ops), max_rounds, C.byref(res), dig.ctypes.data,
                                      pops.ctypes.data, rng.ctypes.data, ev.ctypes.data)
    err = lib.sg_policy_ops_gpu_error(C.byref(ops)) if getattr(ops, "_owner", "") == "gpu" else 0
    if free_ops:
        ops.free(ops.data)
    L.check(rc)
    L.check(err)
    out = res.as_dict()
    out.update(digest=dig, pops_per_host=pops, rng=rng, ev=ev)
    return out
