"""GPU: a seeded sweep of randomly drawn small PHOLD configurations, each run
through the unsharded engine, through 1-3 in-process shards and through the
drop-in `gpu` policy at 1-8 workers, against the CPU
oracle (bit-exact: per-host digests, pop counts, rand_r states, event-id
counters and the global counters).

The fixed cases in test_gpu_parity.py / test_gpu_sharded.py each vary one knob;
this sweep draws all of them together (host count, vertices, load, edge loss,
latency floor, runahead, window rule, destination rule, weights, bootstrap
horizon, end time, queue capacity, exchange capacity) so combinations nobody
wrote down are covered too.  The draws come from numpy's seeded generator, so a
failure names its seed and reproduces exactly."""
import numpy as np
import pytest

from shadow_amd import phold, policy
from shadow_amd import _lib as L
from oracle import oracle as O

from test_gpu_parity import _run_both, _assert_same
from test_gpu_sharded import _run_shards, _check

SEEDS = list(range(101, 125))


def _draw(seed):
    r = np.random.default_rng(seed)
    n = int(r.choice([1, 2, 7, 64, 257, 640, 1500, 4000]))
    V = int(r.integers(1, 9))
    kw = dict(n_hosts=n, V=V, load=int(r.integers(1, 7)), seed=int(r.integers(1, 1 << 30)),
              end_time_s=float(r.choice([0.15, 0.3, 0.6])),
              loss=float(r.choice([0.0, 0.05, 0.3])),
              min_ms=float(r.choice([0.2, 1.0, 3.0])),
              runahead_ms=float(r.choice([0, 0, 2, 9])),
              window_rule=int(r.choice([L.SG_WINDOW_DISCOVERED, L.SG_WINDOW_FIXED])),
              dst_rule=int(r.choice([L.SG_DST_WEIGHTS, L.SG_DST_UNIFORM_FLOOR])))
    if kw["dst_rule"] == L.SG_DST_WEIGHTS and r.random() < 0.5:
        kw["weights"] = r.uniform(0.05, 4.0, n) ** 2
    cfg = phold.tiny_config(**kw)
    if kw["window_rule"] == L.SG_WINDOW_FIXED:
        cfg["fixed_jump"] = int(r.choice([1, 5, 20])) * L.ONE_MS
    if r.random() < 0.3:
        cfg["bootstrap_end"] = int(r.choice([20, 100])) * L.ONE_MS
    queue_cap = int(r.choice([0, 0, 1, 64]))
    world = int(r.integers(1, 4))
    xcap = int(r.choice([7, 64, 4096]))
    return cfg, queue_cap, world, xcap


@pytest.mark.gpu
@pytest.mark.parametrize("seed", SEEDS)
def test_random_config_gpu_policy(seed):
    """The same draws through the drop-in `gpu` SchedulerPolicy (Mode P: CPU
    workers, device queues) under the Shadow-style round driver, at a drawn
    worker count (more workers than hosts included)."""
    cfg, *_ = _draw(seed)
    workers = int(np.random.default_rng(seed + 7).choice([1, 2, 3, 5, 8]))
    ref = O.Sim(cfg)
    ref.boot()
    ref.run()
    rs, st = ref.host_state(), ref.stats()
    r = policy.run_phold(cfg, workers, policy.gpu_ops(workers, cfg["n_hosts"]))
    for k, rk in (("digest", "digest"), ("pops_per_host", "pops"), ("rng", "rng"), ("ev", "ev")):
        assert np.array_equal(r[k], rs[rk]), (seed, workers, k)
    for k in ("rounds", "pops", "sends", "drop_reliability", "drop_endtime", "bumped"):
        assert r[k] == st[k], (seed, workers, k)


LARGE_SEEDS = list(range(201, 209))


def _draw_large(seed):
    """Shard-sized draws: many partitions per launch (and, above 64k hosts, the
    2048-host partition floor), a drawn log-normal topology, a short horizon."""
    r = np.random.default_rng(seed)
    n = int(r.choice([5000, 20_000, 70_000, 150_000]))
    V = int(r.choice([16, 64, 256]))
    lat, el = phold.lognormal_topology(V, int(r.integers(1, 1000)),
                                       median_ms=float(r.uniform(5, 40)),
                                       sigma=float(r.uniform(0.3, 1.0)),
                                       min_ms=float(r.choice([0.5, 1.0, 2.0])),
                                       edge_loss=float(r.choice([0.0, 0.01, 0.1])))
    cfg = phold.make_config(n_hosts=n, latency_ms=lat, edge_loss=el,
                            load=int(r.choice([1, 4, 16])), seed=int(r.integers(1, 1 << 30)),
                            end_time_s=float(r.choice([0.05, 0.1])),
                            runahead_ms=float(r.choice([0, 1, 3])),
                            dst_rule=int(r.choice([L.SG_DST_WEIGHTS, L.SG_DST_UNIFORM_FLOOR])),
                            name=f"sweep-{seed}")
    return cfg, 0, int(r.integers(1, 5)), int(r.choice([256, 1 << 16]))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", SEEDS)
def test_random_config_unsharded(seed):
    cfg, queue_cap, _, _ = _draw(seed)
    eng, orc = _run_both(cfg, queue_cap=queue_cap)
    gs = _assert_same(eng, orc)
    assert gs["pops"] > 0, seed


@pytest.mark.gpu
@pytest.mark.parametrize("seed", SEEDS)
def test_random_config_sharded(seed):
    cfg, _, world, xcap = _draw(seed)
    world = min(world, cfg["n_hosts"])
    shards, _ = _run_shards(cfg, world, xcap)
    _check(cfg, shards)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", LARGE_SEEDS)
def test_random_large_config(seed):
    cfg, _, world, xcap = _draw_large(seed)
    eng, orc = _run_both(cfg)
    gs = _assert_same(eng, orc)
    assert gs["pops"] > 0, seed
    shards, _ = _run_shards(cfg, world, xcap)
    _check(cfg, shards)


def test_draws_cover_the_knobs():
    """The sweep is only worth its time if the draws actually vary the knobs."""
    d = [_draw(s) for s in SEEDS]
    assert len({c["n_hosts"] for c, *_ in d}) >= 4
    assert {c["window_rule"] for c, *_ in d} == {L.SG_WINDOW_DISCOVERED, L.SG_WINDOW_FIXED}
    assert {c["dst_rule"] for c, *_ in d} == {L.SG_DST_WEIGHTS, L.SG_DST_UNIFORM_FLOOR}
    assert any(c["runahead_min"] > 0 for c, *_ in d)
    assert any(c["bootstrap_end"] > 0 for c, *_ in d)
    assert any(q > 0 for _, q, _, _ in d)
    assert {w for *_, w, _ in d} >= {1, 2}
