"""GPU: the drop-in `gpu` SchedulerPolicy (Mode P) — CPU worker threads execute
the events, per-host queues / sort / MIN live in HBM — under the Shadow-style
round driver; per-host traces must equal the oracle's, for any worker count."""
import numpy as np
import pytest

from oracle import oracle as O
from shadow_amd import phold, policy

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kind,workers", [("tiny_lossy", 1), ("tiny_lossy", 4),
                                          ("probe10_bumps", 3), ("c2_small", 8),
                                          ("self_heavy", 2), ("runahead", 5),
                                          ("gossip_small", 1), ("gossip_small", 6)])
def test_gpu_policy_matches_oracle(kind, workers):
    cfg = {
        "tiny_lossy": lambda: phold.tiny_config(n_hosts=200, V=6, load=4, end_time_s=0.4, loss=0.1),
        "probe10_bumps": lambda: phold.probe_config(n_hosts=300, jump_ms=10, end_time_s=0.5),
        "c2_small": lambda: phold.c2_config(n_hosts=2000, end_time_s=0.6),
        # 4 hosts: a quarter of all sends are self events, many inside the window
        "self_heavy": lambda: phold.probe_config(n_hosts=4, jump_ms=20, end_time_s=0.5),
        "runahead": lambda: phold.tiny_config(n_hosts=120, runahead_ms=6, end_time_s=0.3),
        # configs[4]'s gossip body: lossy links, origin self events, seen sets
        "gossip_small": lambda: phold.c5_config(n_hosts=3000, V=16, msgs=24, end_time_s=0.6),
    }[kind]()
    ref = O.Sim(cfg)
    ref.boot()
    ref.run()
    rs, st = ref.host_state(), ref.stats()
    r = policy.run_phold(cfg, workers, policy.gpu_ops(workers, cfg["n_hosts"]))
    assert np.array_equal(r["digest"], rs["digest"])
    assert np.array_equal(r["pops_per_host"], rs["pops"])
    assert np.array_equal(r["rng"], rs["rng"])
    assert np.array_equal(r["ev"], rs["ev"])
    for k in ("rounds", "pops", "sends", "drop_reliability", "drop_endtime", "bumped"):
        assert r[k] == st[k], k


def test_gpu_policy_queue_growth():
    """More events queued per host than the initial HBM slots: the policy grows
    its queues and stays exact."""
    cfg = phold.probe_config(n_hosts=6, jump_ms=5, load=200, end_time_s=0.3)
    ref = O.Sim(cfg)
    ref.boot()
    ref.run()
    r = policy.run_phold(cfg, 2, policy.gpu_ops(2, cfg["n_hosts"]))
    assert np.array_equal(r["digest"], ref.host_state()["digest"])


@pytest.mark.parametrize("shift,chunks,compact", [
    (4, 1024, 64),     # 16 ns buckets: the ring reaches 262 us ahead, nearly every event is far
    (30, 1024, 65536),  # 1.07 s buckets: every round extracts from one straddling bucket
    (22, 1, 64),       # 4 ms buckets of one 1024-record chunk: full buckets overflow to the far list
])
def test_gpu_policy_calendar_paths(monkeypatch, shift, chunks, compact):
    """The device calendar's less common paths stay exact: the far list (beyond
    the ring, or past a full bucket) with its compaction, and tombstones in a
    bucket that straddles every barrier."""
    monkeypatch.setenv("SG_PBUCKET_SHIFT", str(shift))
    monkeypatch.setenv("SG_PBUCKET_CHUNKS", str(chunks))
    monkeypatch.setenv("SG_PFAR_COMPACT", str(compact))
    cfg = phold.c2_config(n_hosts=2000, end_time_s=0.4)
    ref = O.Sim(cfg)
    ref.boot()
    ref.run()
    rs, st = ref.host_state(), ref.stats()
    r = policy.run_phold(cfg, 4, policy.gpu_ops(4, cfg["n_hosts"]))
    assert np.array_equal(r["digest"], rs["digest"])
    assert np.array_equal(r["pops_per_host"], rs["pops"])
    for k in ("rounds", "pops", "sends", "bumped"):
        assert r[k] == st[k], k


def test_gpu_policy_many_host_blocks():
    """50k hosts: the extraction's host sort spans 13 host blocks of 4096 and
    several level-1 units per round."""
    cfg = phold.c2_config(n_hosts=50_000, end_time_s=0.15)
    ref = O.Sim(cfg)
    ref.boot()
    ref.run()
    rs, st = ref.host_state(), ref.stats()
    r = policy.run_phold(cfg, 8, policy.gpu_ops(8, cfg["n_hosts"]))
    assert np.array_equal(r["digest"], rs["digest"])
    assert np.array_equal(r["pops_per_host"], rs["pops"])
    for k in ("rounds", "pops", "sends", "bumped"):
        assert r[k] == st[k], k


@pytest.mark.parametrize("seed,hosts", [(2, 8), (11, 5), (33, 3)])
def test_gpu_policy_ordered_discovery(seed, hosts):
    """Row (f)-2 on the drop-in path: the `gpu` policy under one CPU worker
    (shadow -w 1) on an incomplete graph, every send looked up in the
    reference's lazy path cache in pop order (sg_path_cache), equals the
    oracle's restatement of that cache; source-wide discovery gives another
    run (tests/test_topology_cache_order.py)."""
    from tests.test_topology_cache_order import ordered_case
    runs = {}
    for disc in ("source", "ordered"):
        cfg = ordered_case(seed, hosts, disc)
        ref = O.Sim(cfg)
        ref.boot()
        ref.run()
        st, hs = ref.stats(), ref.host_state()
        r = policy.run_phold(cfg, 1, policy.gpu_ops(1, hosts))
        assert (r["rounds"], r["bumped"], r["pops"]) == (st["rounds"], st["bumped"], st["pops"]), disc
        assert np.array_equal(r["digest"], hs["digest"]) and np.array_equal(r["ev"], hs["ev"]), disc
        runs[disc] = (st["rounds"], st["bumped"])
    assert runs["source"] != runs["ordered"]


@pytest.mark.parametrize("n,w0", [(600, 200.0), (3000, 3000.0)])
def test_gpu_policy_incast(n, w0):
    """one destination receives a large share of every round's events
    (weights rule, host 0 weighted w0).  Runs longer than k_xrank's scan bound
    go to k_xlong: up to 2048 records sorted in LDS (600 hosts: runs up to ~600
    per round), beyond that ranked in LDS tiles (3000 hosts: runs up to ~5400)."""
    w = np.ones(n)
    w[0] = w0
    cfg = phold.tiny_config(n_hosts=n, V=4, load=8, end_time_s=0.3, loss=0.0, weights=w)
    ref = O.Sim(cfg)
    ref.boot()
    ref.run()
    rs, st = ref.host_state(), ref.stats()
    r = policy.run_phold(cfg, 4, policy.gpu_ops(4, cfg["n_hosts"]))
    assert np.array_equal(r["digest"], rs["digest"])
    assert np.array_equal(r["pops_per_host"], rs["pops"])
    assert np.array_equal(r["ev"], rs["ev"])
    for k in ("rounds", "pops", "sends", "bumped"):
        assert r[k] == st[k], k


def test_gpu_policy_kernel_profile():
    """The device half's per-kernel profile (sg_policy_kernel_profile): every
    insert / MIN / extraction kernel class is timed and carries algorithmic
    bytes over the rounds after the skipped ones, and profiling changes nothing
    in the run (per-host state still equals the oracle's)."""
    cfg = phold.c2_config(n_hosts=2000, end_time_s=0.6)
    ref = O.Sim(cfg)
    ref.boot()
    ref.run()
    rs = ref.host_state()
    ops = policy.gpu_ops(3, cfg["n_hosts"])
    try:
        policy.kernel_profile(ops, True, 2)
        r = policy.run_phold(cfg, 3, ops, free_ops=False)
        ks = policy.kernel_stats(ops)
    finally:
        ops.free(ops.data)
    assert np.array_equal(r["digest"], rs["digest"])
    assert list(ks)[:6] == ["k_cins1", "k_cneed", "k_calloc", "k_cins2", "k_cmin", "k_xplan"]
    for k in ("k_cins1", "k_cins2", "k_cmin", "k_xplan", "k_hist", "k_part", "k_local", "k_xrank"):
        assert ks[k]["launches"] > 0 and ks[k]["ms"] > 0 and ks[k]["alg_bytes"] > 0, (k, ks[k])
    # the extraction classes ran once per counted round
    assert ks["k_hist"]["launches"] == ks["k_part"]["launches"] == ks["k_xrank"]["launches"]
    assert ks["k_hist"]["launches"] <= r["rounds"] - 2 + 1
