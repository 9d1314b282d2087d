"""GPU: every BASELINE config on the HIP path at its configured size, against the
CPU oracle (live where it runs in seconds, otherwise the committed fixtures of
tests/golden/oracle_fixtures.json that tests/golden/make_fixtures.py wrote from
the same oracle).

  configs[0] C1  two hosts on the example's embedded one-vertex topology, the
                 whole 3600 s run, through the device engine and through the
                 `gpu` SchedulerPolicy (Mode P) against host_single semantics
  configs[2] C3  2k relays + 8k clients on the bundled topology, 10 s, through
                 the engine (per-host pop-trace diff) and the `gpu` policy with
                 8 and 16 CPU workers
  configs[3] C4  1M hosts: the state after the rounds the bench times
                 (fingerprint per round from the oracle), unsharded and as 8
                 in-process shards of 125k hosts (small exchange blocks, so
                 drain steps occur)
  configs[4] C5  gossip, 100k hosts, lossy links, the whole run: unsharded and
                 with 2 / 4 / 8 in-process shards

Integer work throughout: the bar is bit-exact (fingerprint = checksum of every
host's trace digest, pops, rand_r state and event counter).
"""
import json
import os

import numpy as np
import pytest

from oracle import oracle as O
from shadow_amd import phold, policy
from shadow_amd.engine import Engine
from shadow_amd.trace import state_fingerprint

pytestmark = pytest.mark.gpu
FIX = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "oracle_fixtures.json")))
STATS = ("rounds", "pops", "boots", "sends", "null_dst", "drop_reliability", "drop_endtime",
         "bumped", "same_round", "pending", "done", "jmin_ms")


def _fp(eng):
    hs = eng.host_state()
    return state_fingerprint(eng.first_host, hs["digest"], hs["pops"], hs["rng"], hs["ev"])


def _windows_fp(w):
    h, M = 5381, (1 << 64) - 1
    for s, e in w.tolist():
        h = ((h * 1000003) ^ s) & M
        h = ((h * 1000003) ^ e) & M
    return h


def _check_final(name, eng_stats, fp, windows=None):
    fx = FIX[name]
    for k in STATS:
        assert eng_stats[k] == fx["stats"][k], (name, k, eng_stats[k], fx["stats"][k])
    assert eng_stats["overflow"] == 0
    assert fp == fx["fingerprint"], name
    if windows is not None:
        assert _windows_fp(windows) == fx["windows_fp"], name


# ------------------------------------------------------------------ C1 -----
def test_c1_engine_whole_run():
    cfg = phold.c1_config()
    eng = Engine(cfg, trace_capacity=1 << 16)
    eng.boot()
    eng.run()
    _check_final("c1", eng.stats(), _fp(eng), eng.windows())
    orc = O.Sim(cfg, trace_capacity=1 << 16)
    orc.boot()
    orc.run()
    key = ["host", "pos"]
    assert np.array_equal(np.sort(eng.trace(), order=key), np.sort(orc.trace(), order=key))


@pytest.mark.parametrize("workers", [1, 2])
def test_c1_gpu_policy_whole_run(workers):
    """The drop-in `gpu` SchedulerPolicy on configs[0] against the oracle's
    host_single semantics (host_single.c:167-305) and the threaded host_single
    restatement under the same round driver."""
    cfg = phold.c1_config()
    r = policy.run_phold(cfg, workers, policy.gpu_ops(workers, cfg["n_hosts"]))
    fp = state_fingerprint(0, r["digest"], r["pops_per_host"], r["rng"], r["ev"])
    assert fp == FIX["c1"]["fingerprint"]
    for k in ("rounds", "pops", "sends", "drop_reliability", "drop_endtime", "bumped"):
        assert r[k] == FIX["c1"]["stats"][k], k
    hs = policy.run_phold(cfg, workers, O.cpu_policy_ops(False, workers, cfg["n_hosts"]))
    assert np.array_equal(hs["digest"], r["digest"])


# ------------------------------------------------------------------ C3 -----
def test_c3_engine_full_size_trace_diff():
    from shadow_amd import trace as T
    cfg = phold.c3_config()
    assert cfg["n_hosts"] == 10_000
    eng = Engine(cfg, trace_capacity=4_000_000)
    eng.boot()
    eng.run()
    _check_final("c3", eng.stats(), _fp(eng), eng.windows())
    orc = O.Sim(cfg, trace_capacity=4_000_000)
    orc.boot()
    orc.run()
    d = T.diff(eng.trace(), orc.trace())
    assert d["identical"] and d["pops_a"] == FIX["c3"]["stats"]["pops"]


@pytest.mark.parametrize("workers", [8, 16])
def test_c3_gpu_policy_full_size(workers):
    cfg = phold.c3_config()
    r = policy.run_phold(cfg, workers, policy.gpu_ops(workers, cfg["n_hosts"]))
    fp = state_fingerprint(0, r["digest"], r["pops_per_host"], r["rng"], r["ev"])
    assert fp == FIX["c3"]["fingerprint"]
    for k in ("rounds", "pops", "sends", "drop_reliability", "drop_endtime", "bumped"):
        assert r[k] == FIX["c3"]["stats"][k], k


# ------------------------------------------------------------------ C4 -----
C4_CHECK = (1, 2, 25, 220, 270, 600)


def test_c4_1m_bench_rounds_pinned():
    """The rounds behind the headline number: the 1M-host state after each
    checked round equals the oracle's (the bench's default region is rounds
    21-220, then 50 k_proc-timed and 50 all-timed rounds; the driver's 6-25)."""
    rows = {r[0]: r for r in FIX["c4_1m"]["rounds"]}
    eng = Engine(phold.c4_config(n_hosts=1_000_000))
    eng.boot()
    done = 0
    for r in C4_CHECK:
        eng.run(r - done)
        done = r
        st = eng.stats()
        assert st["rounds"] == r and st["overflow"] == 0
        assert st["pops"] == rows[r][1], r
        assert (st["window_start"], st["window_end"]) == (rows[r][3], rows[r][4]), r
        assert _fp(eng) == rows[r][2], r


def _run_inprocess(cfg, world, xcap, until_round=None, queue_cap=0):
    import torch
    from shadow_amd.dist import EngineShard
    stream = torch.cuda.Stream()
    shards = [EngineShard(cfg, r, world, 0, exchange_cap=xcap, stream=stream, queue_cap=queue_cap)
              for r in range(world)]
    steps = 0
    with torch.cuda.stream(stream):
        for s in shards:
            s.boot()
        while True:
            sends = [s.pre() for s in shards]
            for r, s in enumerate(shards):  # all_to_all_single: block r of every sender
                for p in range(world):
                    s.recv[p].copy_(sends[p][r])
            for s in shards:
                s.post()
            steps += 1
            if steps % 8 == 0 or until_round is not None:
                st = shards[0].stats()
                if st["done"] or (until_round is not None and st["rounds"] >= until_round
                                  and st["phase"] == 0):
                    break
            assert steps < 400_000
    stream.synchronize()
    return shards, steps


def test_c4_1m_eight_shards():
    """configs[3]'s 8-way split (125k hosts per shard) through the step protocol
    the 8-GPU bench runs, exchange blocks of 4096 rows (the boot round and the
    steady rounds drain over extra steps), against the oracle at round 40."""
    rows = {r[0]: r for r in FIX["c4_1m"]["rounds"]}
    cfg = phold.c4_config(n_hosts=1_000_000)
    shards, steps = _run_inprocess(cfg, 8, 4096, until_round=40)
    st = [s.stats() for s in shards]
    assert all(x["overflow"] == 0 for x in st), [hex(x["overflow"]) for x in st]
    assert all(x["rounds"] == 40 for x in st)
    assert steps > 40  # drain steps happened
    assert sum(x["pops"] for x in st) == rows[40][1]
    fp = sum(s.fingerprint() for s in shards) & ((1 << 64) - 1)
    assert fp == rows[40][2]
    for x in st:
        assert (x["window_start"], x["window_end"]) == (rows[40][3], rows[40][4])


# ------------------------------------------------------------------ C5 -----
def test_c5_gossip_whole_run_unsharded():
    cfg = phold.c5_config()
    assert cfg["n_hosts"] == 100_000
    eng = Engine(cfg)
    eng.boot()
    eng.run()
    st = eng.stats()
    _check_final("c5", st, _fp(eng))
    assert st["drop_reliability"] > 0
    oc = eng.object_counts()
    assert oc["event_new"] - oc["event_free"] == oc["event_live"] == 0


@pytest.mark.parametrize("world", [2, 4, 8])
def test_c5_gossip_whole_run_shards(world):
    cfg = phold.c5_config()
    shards, steps = _run_inprocess(cfg, world, 8192)
    st = [s.stats() for s in shards]
    assert all(x["overflow"] == 0 for x in st), [hex(x["overflow"]) for x in st]
    fx = FIX["c5"]["stats"]
    for k in ("pops", "boots", "sends", "drop_reliability", "drop_endtime", "bumped", "same_round"):
        assert sum(x[k] for x in st) == fx[k], k
    for x in st:
        assert x["rounds"] == fx["rounds"] and x["done"]
    fp = sum(s.fingerprint() for s in shards) & ((1 << 64) - 1)
    assert fp == FIX["c5"]["fingerprint"]
