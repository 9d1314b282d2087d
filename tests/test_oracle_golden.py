"""CPU: the oracle against every golden vector available for this path.

* the reference-produced trace hashes recorded by the survey (the reference's
  own scheduler.c + policies driven by a PHOLD harness): window = min latency
  (serial == host_single == host_steal) and window 10 ms (bump visible);
* glibc's own rand_r (the third-party dependency, present in this image);
* SURVEY.md Appendix A known answers (seed chain, ceil delays, truncation).
"""
import ctypes
import ctypes.util
import json
import math
import os

import numpy as np
import pytest

from oracle import oracle as O
from shadow_amd import phold

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
KAT = json.load(open(os.path.join(GOLDEN, "kat.json")))
PROBE = json.load(open(os.path.join(GOLDEN, "probe_hashes.json")))


def _libc():
    return ctypes.CDLL(ctypes.util.find_library("c"))


@pytest.mark.parametrize("seed", [0, 1, 2, 12345, 0x7FFFFFFF, 0xFFFFFFFF, 3141592653])
def test_oracle_rand_r_is_glibc(seed):
    libc = _libc()
    libc.rand_r.argtypes = [ctypes.POINTER(ctypes.c_uint)]
    st = ctypes.c_uint(seed)
    want = [libc.rand_r(ctypes.byref(st)) for _ in range(2000)]
    assert O.rand_r_stream(seed, 2000).tolist() == want


def test_rand_r_kat():
    assert O.rand_r_stream(1, 5).tolist() == KAT["rand_r_seed1_first5"]


def test_seed_chain_kat():
    a, b, node = O.seed_chain(1, 4)
    k = KAT["seed_chain_s1"]
    assert (a, b) == (k["slave_seed"], k["scheduler_seed"])
    assert node.tolist() == k["host_seeds_first4"]


def test_delay_and_truncation_kats():
    lat = np.array([x for x, _ in KAT["ceil_delay_ns"]])
    d, k, j = O.build_paths(np.diag(lat).ravel() if len(lat) > 1 else lat, np.zeros(len(lat) ** 2))
    V = len(lat)
    for i, (_, ns) in enumerate(KAT["ceil_delay_ns"]):
        assert int(d[i * V + i]) == ns
    (ms, tr), = KAT["trunc_ms"]
    d2, _, j2 = O.build_paths(np.array([ms]), np.zeros(1))
    assert int(j2[0]) == tr
    assert int(d2[0]) == math.ceil(ms * 1e6)


def _probe_cfg(jump):
    # the probe's tables are built independently of the product here
    V = 8
    _, _, node = O.seed_chain(1, 1000)
    vert, rng = O.attach(node, V, 0)
    delay = np.array([math.ceil((5.0 + 3.37 * ((i * 7 + j * 3) % V)) * 1000000)
                      for i in range(V) for j in range(V)], np.uint64)
    rel = 0.99
    lo, hi = 0, 2147483647
    while hi - lo > 1:
        m = (lo + hi) // 2
        lo, hi = (m, hi) if m / 2147483647 <= rel else (lo, m)
    return dict(n_hosts=1000, n_vertices=V, load=16, dst_rule=0, window_rule=0,
                end_time=2_000_000_000, fixed_jump=jump * 1_000_000, host_vertex=vert,
                host_rng=rng, delay_ns=delay, keep_max=np.full(V * V, lo, np.int32),
                jump_ms=np.full(V * V, 5, np.uint32))


@pytest.mark.parametrize("jump", [5, 10])
def test_oracle_reproduces_reference_probe_hash(jump):
    gold = PROBE[f"jump_{jump}ms"]
    s = O.Sim(_probe_cfg(jump), trace_capacity=1_300_000)
    s.boot()
    s.run()
    h, n = s.probe_hash()
    assert n == gold["messages"]
    assert f"{h:016x}" == gold["hash"]


def test_serial_policy_equals_rounds_when_window_is_min_latency():
    """global_single (-w 0) and the host policies agree when the window equals the
    minimum latency (survey finding 2), and disagree at 10 ms."""
    gold5 = PROBE["jump_5ms"]
    s = O.Sim(_probe_cfg(5), mode=O.MODE_SERIAL, trace_capacity=1_300_000)
    s.boot()
    s.run_serial()
    h, n = s.probe_hash()
    assert (f"{h:016x}", n) == (gold5["hash"], gold5["messages"])
    assert PROBE["jump_10ms"]["hash"] != gold5["hash"]


def test_product_probe_config_matches_oracle_tables():
    """shadow_amd.phold builds the probe's tables with libshadowgpu host code;
    they must equal the oracle's independent construction."""
    cfg = phold.probe_config(n_hosts=1000, jump_ms=5)
    ref = _probe_cfg(5)
    for k in ("host_vertex", "host_rng", "delay_ns", "keep_max"):
        assert np.array_equal(np.asarray(cfg[k]), np.asarray(ref[k])), k
