"""CPU: the round driver (sg_sched.c, scheduler.c/worker.c restated) with real
worker threads under the host_single / host_steal restatements reproduces the
oracle's per-host traces for any worker count (survey finding 2: per-host
traces do not depend on worker count or host->thread assignment)."""
import numpy as np
import pytest

from oracle import oracle as O
from shadow_amd import phold, policy


def _cases():
    return {
        "tiny_lossy": lambda: phold.tiny_config(n_hosts=200, V=6, load=4, end_time_s=0.4, loss=0.1),
        "probe10_bumps": lambda: phold.probe_config(n_hosts=300, jump_ms=10, end_time_s=0.5),
        "c2_small": lambda: phold.c2_config(n_hosts=500, end_time_s=0.6),
        "runahead": lambda: phold.tiny_config(n_hosts=120, runahead_ms=6, end_time_s=0.3),
        # configs[4]'s gossip body under the CPU workers (sg_sched.c)
        "gossip_small": lambda: phold.c5_config(n_hosts=3000, V=16, msgs=24, end_time_s=0.6),
    }


@pytest.mark.parametrize("kind", list(_cases()))
@pytest.mark.parametrize("steal,workers", [(False, 1), (False, 4), (True, 2), (True, 8)])
def test_threaded_cpu_policy_matches_oracle(kind, steal, workers):
    cfg = _cases()[kind]()
    ref = O.Sim(cfg)
    ref.boot()
    ref.run()
    rs, st = ref.host_state(), ref.stats()
    r = policy.run_phold(cfg, workers, O.cpu_policy_ops(steal, workers, cfg["n_hosts"]))
    assert np.array_equal(r["digest"], rs["digest"])
    assert np.array_equal(r["pops_per_host"], rs["pops"])
    assert np.array_equal(r["rng"], rs["rng"])
    assert np.array_equal(r["ev"], rs["ev"])
    for k in ("rounds", "pops", "sends", "drop_reliability", "drop_endtime", "bumped"):
        assert r[k] == st[k], k


@pytest.mark.parametrize("kind", ["tiny_lossy", "c2_small", "gossip_small"])
@pytest.mark.parametrize("steal,workers", [(False, 1), (True, 4)])
def test_faithful_heap_policy_matches_oracle(kind, steal, workers):
    """The faithful CPU baseline (oracle/libhsglib.so: priority_queue.c's heap
    with its GLib hash-table position map under the same host_steal /
    host_single restatement) pops the same per-host sequences."""
    if not O.faithful_available():
        pytest.skip("GLib headers absent: libhsglib.so not built")
    cfg = _cases()[kind]()
    ref = O.Sim(cfg)
    ref.boot()
    ref.run()
    rs, st = ref.host_state(), ref.stats()
    r = policy.run_phold(cfg, workers, O.cpu_policy_ops(steal, workers, cfg["n_hosts"], faithful=True))
    for k in ("digest", "rng", "ev"):
        assert np.array_equal(r[k], rs[k]), k
    assert np.array_equal(r["pops_per_host"], rs["pops"])
    for k in ("rounds", "pops", "sends", "drop_reliability", "drop_endtime", "bumped"):
        assert r[k] == st[k], k
