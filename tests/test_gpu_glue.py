"""The Shadow-side glue (integration/scheduler_policy_gpu.c) linked to the REAL
libshadowgpu.so, driven through its SchedulerPolicy vtable (scheduler_policy.h:
31-58) by the library's Shadow-style round driver (scheduler.c:339-414,
617-650; worker.c:149-216), with test doubles only for Host / Event / Options /
the logger (tests/glue_phold.c).  Per-host digests, pop counts, RNG states,
event counters and the driver's counters must equal the oracle's.

The glue libraries (integration/_bin/libsgglue_{relabel,exact}.so) are compiled
against the reference's own headers by __graft_entry__.build() in the build
container and travel to the GPU box with the tree."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

from oracle import oracle as O
from shadow_amd import _lib as L
from shadow_amd import build as B
from shadow_amd import phold, policy

VARIANTS = ("relabel", "exact")


class GlueReport(C.Structure):
    _fields_ = [(n, C.c_int64) for n in ("live_after_free", "unref_at_free", "errors", "exact_ids")]


def _glue_path(variant):
    return os.path.join(B.GLUE_BIN, f"libsgglue_{variant}.so")


def _need_glue(variant):
    path = _glue_path(variant)
    if not os.path.exists(path):
        if B.glue_available():
            pytest.fail(f"{path} missing: run __graft_entry__.build()")
        pytest.skip("glue not built: it needs the reference headers (build container) and was not shipped")
    if not os.path.exists(os.path.join(B.GLIB_LIB, "libglib-2.0.so.0")):
        pytest.skip(f"GLib ({B.GLIB_LIB}/libglib-2.0.so.0) absent on this machine: the glue cannot load")
    return path


_loaded = {}


def _glue(variant):
    if variant not in _loaded:
        L.lib()  # the product library first: the glue's DT_NEEDED resolves to this same object
        g = C.CDLL(_need_glue(variant))
        g.glue_run_phold.argtypes = [C.POINTER(L.PholdParams), C.POINTER(L.PholdTables), C.c_uint32,
                                     C.c_uint32, C.c_uint64, C.POINTER(policy.SchedResult), C.c_void_p,
                                     C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(GlueReport)]
        _loaded[variant] = g
    return _loaded[variant]


def run_glue(cfg, variant, n_workers, max_rounds=1 << 62):
    g = _glue(variant)
    p, t, _keep = policy.phold_args(cfg)
    n = cfg["n_hosts"]
    dig, pops, ev = (np.zeros(n, np.uint64) for _ in range(3))
    rng = np.zeros(n, np.uint32)
    res, rep = policy.SchedResult(), GlueReport()
    rc = g.glue_run_phold(C.byref(p), C.byref(t), n_workers, policy.default_scheduler_seed(cfg), max_rounds,
                          C.byref(res), dig.ctypes.data, pops.ctypes.data, rng.ctypes.data, ev.ctypes.data,
                          C.byref(rep))
    L.check(rc)
    out = res.as_dict()
    out.update(digest=dig, pops_per_host=pops, rng=rng, ev=ev,
               report={n: int(getattr(rep, n)) for n, _ in GlueReport._fields_})
    return out


def _oracle(cfg, max_rounds=1 << 62):
    ref = O.Sim(cfg)
    ref.boot()
    ref.run(max_rounds)
    return ref.host_state(), ref.stats()


def _assert_same(r, hs, st):
    assert np.array_equal(r["digest"], hs["digest"])
    assert np.array_equal(r["pops_per_host"], hs["pops"])
    assert np.array_equal(r["rng"], hs["rng"])
    assert np.array_equal(r["ev"], hs["ev"])
    for k in ("rounds", "pops", "sends", "drop_reliability", "drop_endtime", "bumped"):
        assert r[k] == st[k], k


@pytest.mark.parametrize("variant", VARIANTS)
def test_glue_links_real_library(variant):
    """CPU: the glue library exists, loads, and takes every sg_policy_* from
    libshadowgpu.so (undefined in the glue, defined by the product library):
    nothing in it stands in for the product."""
    path = _need_glue(variant)
    nm = subprocess.run(["nm", "-D", path], capture_output=True, text=True, check=True).stdout
    syms = {ln.split()[-1]: ln.split()[-2] for ln in nm.splitlines() if len(ln.split()) >= 2}
    for s in ("sg_policy_create", "sg_policy_add_host", "sg_policy_thread_hosts", "sg_policy_push",
              "sg_policy_pop", "sg_policy_next_time", "sg_policy_remaining", "sg_policy_destroy",
              "sg_sched_run_phold"):
        assert syms.get(s) == "U", s
    assert syms.get("schedulerpolicygpu_new") == "T"
    assert syms.get("glue_run_phold") == "T"
    needed = subprocess.run(["readelf", "-d", path], capture_output=True, text=True, check=True).stdout
    assert "[libshadowgpu.so]" in needed and "[libglib-2.0.so.0]" in needed
    _glue(variant)  # loads (no GPU call)


@pytest.mark.gpu
@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("kind,workers", [("tiny_lossy", 1), ("tiny_lossy", 4), ("probe10_bumps", 4),
                                          ("self_heavy", 1)])
def test_glue_phold_matches_oracle(variant, kind, workers):
    """PHOLD through schedulerpolicygpu_new()'s vtable on the real library:
    the glue's GQuark → index map, its once-only creation after addHost, the
    srcHostEventID relabelling (or the exact getter) and free's unref drain."""
    cfg = {
        "tiny_lossy": lambda: phold.tiny_config(n_hosts=200, V=6, load=4, end_time_s=0.4, loss=0.1),
        "probe10_bumps": lambda: phold.probe_config(n_hosts=300, jump_ms=10, end_time_s=0.5),
        "self_heavy": lambda: phold.probe_config(n_hosts=4, jump_ms=20, end_time_s=0.5),
    }[kind]()
    hs, st = _oracle(cfg)
    r = run_glue(cfg, variant, workers)
    _assert_same(r, hs, st)
    rep = r["report"]
    assert rep["exact_ids"] == (variant == "exact")
    assert rep["errors"] == 0
    assert rep["live_after_free"] == 0
    assert rep["unref_at_free"] == st["pending"]  # whatever the run left queued, free unrefs


@pytest.mark.gpu
@pytest.mark.parametrize("variant", VARIANTS)
def test_glue_idle_worker(variant):
    """Three workers, two hosts: the third worker owns no host but
    still calls getNextTime every round (scheduler.c:393-394), so the policy is
    sized from the scheduler's nWorkers (options_getNWorkerThreads), not from
    the threads addHost named; sized from those it would hang at the first
    round's flush."""
    cfg = phold.probe_config(n_hosts=2, jump_ms=10, load=8, end_time_s=0.3)
    hs, st = _oracle(cfg)
    r = run_glue(cfg, variant, 3)
    _assert_same(r, hs, st)
    assert r["report"]["errors"] == 0 and r["report"]["live_after_free"] == 0


@pytest.mark.gpu
@pytest.mark.parametrize("variant", VARIANTS)
def test_glue_free_unrefs_queued(variant):
    """Stopped after 12 rounds with events still queued in HBM, the CPU heaps
    and the staging arenas: the glue's free unrefs exactly those (host_single.c:
    104 through sg_policy_remaining), no Event reference leaks."""
    cfg = phold.tiny_config(n_hosts=300, V=6, load=6, end_time_s=2.0, loss=0.05)
    hs, st = _oracle(cfg, max_rounds=12)
    r = run_glue(cfg, variant, 4, max_rounds=12)
    _assert_same(r, hs, st)
    rep = r["report"]
    assert st["pending"] > 0
    assert rep["unref_at_free"] == st["pending"]
    assert rep["live_after_free"] == 0 and rep["errors"] == 0
