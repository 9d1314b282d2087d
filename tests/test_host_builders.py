"""CPU: libshadowgpu's host-side restatements (the product's table builders)
against glibc, the oracle's independent restatements and edge cases."""
import ctypes
import ctypes.util
import math

import numpy as np
import pytest

from oracle import oracle as O
from shadow_amd import _lib as L
from shadow_amd import phold


def test_rand_r_matches_glibc_and_oracle():
    libc = ctypes.CDLL(ctypes.util.find_library("c"))
    libc.rand_r.argtypes = [ctypes.POINTER(ctypes.c_uint)]
    for seed in (0, 1, 99, 0xDEADBEEF, 0xFFFFFFFF):
        st = ctypes.c_uint(seed)
        want = [libc.rand_r(ctypes.byref(st)) for _ in range(500)]
        assert phold.rand_r_stream(seed, 500).tolist() == want
        assert O.rand_r_stream(seed, 500).tolist() == want


def test_next_uint_and_double():
    st = ctypes.c_uint32(1)
    st2 = ctypes.c_uint32(1)
    for _ in range(100):
        d = L.lib().sg_random_next_double(ctypes.byref(st))
        r = L.lib().sg_rand_r(ctypes.byref(st2))
        assert d == r / 2147483647.0
    st = ctypes.c_uint32(7)
    st2 = ctypes.c_uint32(7)
    for _ in range(100):
        u = L.lib().sg_random_next_uint(ctypes.byref(st))
        r = L.lib().sg_rand_r(ctypes.byref(st2))
        assert u == int((r / 2147483647.0) * 4294967295.0)


@pytest.mark.parametrize("seed,n", [(1, 5000), (42, 100), (0, 10)])
def test_seed_chain_matches_oracle(seed, n):
    assert [x if isinstance(x, int) else x.tolist() for x in phold.seed_chain(seed, n)] == \
           [x if isinstance(x, int) else x.tolist() for x in O.seed_chain(seed, n)]


@pytest.mark.parametrize("V,rule", [(1, 1), (8, 1), (183, 1), (1024, 1), (8, 0)])
def test_attach_matches_oracle(V, rule):
    _, _, node = phold.seed_chain(1, 3000)
    a = phold.attach(node, V, rule)
    b = O.attach(node, V, rule)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    assert a[0].max() < V
    if rule == 1:  # one draw consumed
        st = ctypes.c_uint32(int(node[0]))
        L.lib().sg_rand_r(ctypes.byref(st))
        assert st.value == a[1][0]


def _thresh_py(c):
    R = 2147483647
    best = -1
    lo, hi = 0, R
    if not (0 / R <= c):
        return -1
    if R / R <= c:
        return R
    while hi - lo > 1:
        m = (lo + hi) // 2
        lo, hi = (m, hi) if m / R <= c else (lo, m)
    return lo


@pytest.mark.parametrize("rel", [0.0, 1e-12, 0.005, 0.5, 0.99, 0.995, 0.999999, 1.0, 1.5, -0.1])
def test_keep_threshold_exact(rel):
    t = phold.keep_threshold(rel)
    assert t == _thresh_py(rel)
    R = 2147483647
    if 0 <= t < R:
        assert t / R <= rel and not ((t + 1) / R <= rel)


def test_build_paths_matches_oracle_and_reference_arithmetic():
    rs = np.random.default_rng(3)
    V = 37
    lat = np.round(rs.uniform(0.5, 2500, V * V), 3)
    el = rs.uniform(0, 0.1, V * V)
    vl = rs.uniform(0, 0.02, V)
    a = phold.build_paths(lat, el, vl)
    b = O.build_paths(lat, el, vl)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
    d, k, j = a
    for i in range(0, V * V, 97):
        s, t = divmod(i, V)
        rel = ((1.0 * (1.0 - vl[s])) * (1.0 - vl[t])) * (1.0 - el[i])
        assert int(d[i]) == math.ceil(lat[i] * 1e6)
        assert int(k[i]) == _thresh_py(rel)
        assert int(j[i]) == int(lat[i])


def test_build_paths_rejects_nonpositive_latency():
    with pytest.raises(L.SgError):
        phold.build_paths(np.array([0.0]), np.zeros(1))


@pytest.mark.parametrize("n,kind", [(10, "ones"), (1000, "ones"), (9, "phold_test"),
                                    (500, "skew"), (64, "zeros_some")])
def test_weight_thresholds(n, kind):
    w = {"ones": np.ones(n), "phold_test": np.full(n, 0.1),
         "skew": np.linspace(0.01, 3, n) ** 3,
         "zeros_some": np.where(np.arange(n) % 3 == 0, 0.0, 1.0)}[kind]
    a = phold.weight_thresholds(w)
    assert np.array_equal(a, O.weight_thresholds(w))
    assert np.all(np.diff(a.astype(np.int64)) >= 0)
    # restated selection == the plugin's loop (test_phold.c:160-178) on sampled draws
    total = 0.0
    for x in w:
        total += x
    rs = np.random.default_rng(n)
    xs = list(rs.integers(0, 2147483648, 300)) + [0, 2147483647]
    for x in xs:
        r = x / 2147483647.0
        cum = 0.0
        want = None
        for i, wi in enumerate(w):
            cum += wi / total
            if cum >= r:
                want = i
                break
        idx = np.nonzero(x <= a.astype(np.int64))[0]
        got = int(idx[0]) if idx.size else None
        assert got == want


def test_window_logic():
    st = L.WindowState(0, 0, 0, 10_000_000_000)
    s, e = ctypes.c_uint64(), ctypes.c_uint64()
    # undiscovered: default 10 ms jump (master.c:137)
    assert L.lib().sg_window_next(ctypes.byref(st), 5, ctypes.byref(s), ctypes.byref(e)) == 1
    assert (s.value, e.value) == (5, 5 + 10_000_000)
    # discovery applies at the next boundary, truncated to whole ms (master.c:153, 459)
    L.lib().sg_window_note_latency(ctypes.byref(st), 47.82)
    assert st.next_min_jump == 47_000_000
    L.lib().sg_window_next(ctypes.byref(st), 100, ctypes.byref(s), ctypes.byref(e))
    assert e.value == 100 + 47_000_000
    # -r lower bound
    st2 = L.WindowState(0, 2_000_000, 5_000_000, 10_000_000_000)
    L.lib().sg_window_next(ctypes.byref(st2), 0, ctypes.byref(s), ctypes.byref(e))
    assert e.value == 5_000_000
    # clamp to endTime and stop when start >= end
    assert L.lib().sg_window_next(ctypes.byref(st), 10_000_000_000, ctypes.byref(s), ctypes.byref(e)) == 0
    # empty queues: SIMTIME_MAX + jump wraps exactly like the reference
    L.lib().sg_window_next(ctypes.byref(st), (1 << 64) - 2, ctypes.byref(s), ctypes.byref(e))
    assert e.value == ((1 << 64) - 2 + 47_000_000) % (1 << 64)
    # sub-millisecond minimum truncates to 0 → back to the 10 ms default
    L.lib().sg_window_note_latency(ctypes.byref(st), 0.4)
    L.lib().sg_window_next(ctypes.byref(st), 0, ctypes.byref(s), ctypes.byref(e))
    assert e.value == 10_000_000


def test_lognormal_topology_symmetric_and_bounded():
    lat, el = phold.lognormal_topology(64, 11, 30.0, 0.9, 1.0, 0.01)
    m = lat.reshape(64, 64)
    assert np.array_equal(m, m.T)
    assert m.min() >= 1.0
    assert np.all(el == 0.01)
