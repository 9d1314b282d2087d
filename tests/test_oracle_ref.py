"""CPU: the oracle and the product's host-side builders against the reference's
own compiled code (oracle/_ref/libshdref.so = utility/random.c +
utility/priority_queue.c from /root/reference, unmodified; `make -C oracle
ref`, run by __graft_entry__.build()).  Skipped where the library was not
built (a checkout without /root/reference).

* random_rand / random_nextDouble / random_nextUInt streams (random.c:32-51)
  against the product's sg_rand_r / sg_random_next_double / sg_random_next_uint
  and the oracle's rand_r;
* the seed chain (master.c:95, 417; slave.c:182, 198, 301) and the attachment
  draw (topology.c:2327-2333) against the product's sg_seed_chain /
  sg_attach_hosts and the oracle's;
* whole PHOLD runs of oracle/refsim.py — the reference's Random per host and
  its PriorityQueue per host, with the reference's floating-point send rules —
  against the oracle: per-host trace digests, pop counts, RNG states, event
  counters, every counter and the final window.

The scheduler itself (scheduler.c, event.c, the policies) is not built: it
needs the simulator's Host/Worker/logger symbols, so parity
stays "partial" beyond what these pin.
"""
import ctypes as C

import numpy as np
import pytest

from oracle import oracle as O
from oracle import refsim
from shadow_amd import _lib as L
from shadow_amd import phold

pytestmark = pytest.mark.skipif(not refsim.available(), reason="oracle/_ref not built")


@pytest.mark.parametrize("seed", [0, 1, 2, 12345, 0x7FFFFFFF, 0xFFFFFFFF, 3141592653])
def test_random_streams_match_reference(seed):
    lib = L.lib()
    r = refsim.Random(seed)
    st = C.c_uint32(seed)
    for _ in range(500):
        assert lib.sg_rand_r(C.byref(st)) == r.rand()
    assert st.value == r.state
    lib.sg_random_next_double.restype = C.c_double
    for _ in range(500):
        assert lib.sg_random_next_double(C.byref(st)) == r.next_double()
    for _ in range(500):
        assert lib.sg_random_next_uint(C.byref(st)) == r.next_uint()
    assert st.value == r.state
    r.free()
    r = refsim.Random(seed)
    assert O.rand_r_stream(seed, 300).tolist() == [r.rand() for _ in range(300)]
    r.free()


@pytest.mark.parametrize("seed", [1, 2, 977])
def test_seed_chain_and_attachment_match_reference(seed):
    n, V = 500, 37
    a, b, node = refsim.seed_chain(seed, n)
    pa, pb, pnode = phold.seed_chain(seed, n)
    oa, ob, onode = O.seed_chain(seed, n)
    assert (a, b) == (pa, pb) == (oa, ob)
    assert node == pnode.tolist() == onode.tolist()
    vert, rng = phold.attach(pnode, V, L.SG_ATTACH_RANDOM)
    for i in range(n):
        r = refsim.Random(node[i])
        rd = r.next_double()
        assert vert[i] == int(refsim._libm.round(float((V - 1) * rd))), i
        assert rng[i] == r.state, i
        r.free()


def _cfg_and_ref(n_hosts, V, *, load, loss, end_s, runahead_ms=0, weights=None, seed=1,
                 min_ms=1.0, bootstrap_end=0):
    lat, el = phold.lognormal_topology(V, seed + 100, median_ms=10.0, sigma=0.8, min_ms=min_ms,
                                       edge_loss=loss)
    cfg = phold.make_config(n_hosts=n_hosts, latency_ms=lat, edge_loss=el, load=load, seed=seed,
                            end_time_s=end_s, runahead_ms=runahead_ms, weights=weights,
                            bootstrap_end=bootstrap_end)
    rel = [1.0 * (1.0 - e) for e in el.tolist()]  # topology.c:1886-1921, no vertex loss
    ref = refsim.RefPhold(n_hosts, lat, rel, load=load, seed=seed, end_time=cfg["end_time"],
                          runahead_ms=runahead_ms, weights=weights, bootstrap_end=bootstrap_end)
    return cfg, ref


@pytest.mark.parametrize("kind", ["lossy", "runahead", "weights", "bootstrap"])
def test_reference_queue_and_rng_run_matches_oracle(kind):
    kw = {"lossy": dict(n_hosts=60, V=6, load=4, loss=0.1, end_s=0.4),
          "runahead": dict(n_hosts=48, V=5, load=3, loss=0.02, end_s=0.3, runahead_ms=4, min_ms=0.3),
          "weights": dict(n_hosts=50, V=4, load=4, loss=0.05, end_s=0.3,
                          weights=np.random.default_rng(3).uniform(0.1, 3.0, 50)),
          "bootstrap": dict(n_hosts=40, V=4, load=4, loss=0.3, end_s=0.3, bootstrap_end=60_000_000)}[kind]
    cfg, ref = _cfg_and_ref(**kw)
    ref.boot()
    ref.run()
    orc = O.Sim(cfg)
    orc.boot()
    orc.run()
    rs, os_ = ref.host_state(), orc.host_state()
    for k in ("digest", "pops", "rng", "ev"):
        assert np.array_equal(rs[k], os_[k]), k
    st = orc.stats()
    for k, v in ref.stats.items():
        assert v == st[k], (k, v, st[k])
    assert (ref.S, ref.E) == (st["window_start"], st["window_end"])
    assert ref.stats["pops"] > 1000
    if kind in ("lossy", "bootstrap"):
        assert ref.stats["drop_reliability"] > 0
    ref.close()
