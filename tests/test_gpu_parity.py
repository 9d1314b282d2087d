"""GPU parity: the HIP round engine against the CPU oracle on identical inputs.

Bit-exact bar: per-host trace digests (order-sensitive over every pop's
(time, src, srcHostEventID)), per-host pop counts, final rand_r states and
event-id counters, the global counters and the window sequence's end state.
Full traces are compared record by record where they are small.
"""
import json
import os

import numpy as np
import pytest

from shadow_amd import phold
from shadow_amd import _lib as L
from shadow_amd.engine import Engine, probe_hash
from oracle import oracle as O

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _run_both(cfg, trace=0, max_rounds=1 << 62, queue_cap=0):
    eng = Engine(cfg, trace_capacity=trace, queue_cap=queue_cap)
    eng.boot()
    eng.run(max_rounds)
    orc = O.Sim(cfg, trace_capacity=trace)
    orc.boot()
    orc.run(max_rounds)
    return eng, orc


def _assert_same(eng, orc):
    g, o = eng.host_state(), orc.host_state()
    for k in ("pops", "rng", "ev", "digest"):
        bad = np.nonzero(g[k] != o[k])[0]
        assert bad.size == 0, f"{k} differs at hosts {bad[:8]}"
    gs, os_ = eng.stats(), orc.stats()
    for k in ("rounds", "pops", "boots", "sends", "null_dst", "drop_reliability",
              "drop_endtime", "bumped", "same_round", "pending", "window_start", "window_end",
              "done", "jmin_ms"):
        assert gs[k] == os_[k], (k, gs[k], os_[k])
    assert gs["overflow"] == 0
    return gs


@pytest.mark.parametrize("jump", [5, 10])
def test_probe_trace_hash_matches_reference(jump):
    """The survey ran the reference's own scheduler.c + host_single/host_steal on
    this workload and recorded these trace hashes (tests/golden/probe_hashes.json)."""
    gold = json.load(open(os.path.join(GOLDEN, "probe_hashes.json")))[f"jump_{jump}ms"]
    cfg = phold.probe_config(n_hosts=1000, jump_ms=jump)
    eng = Engine(cfg, trace_capacity=1_300_000)
    eng.boot()
    eng.run()
    tr = eng.trace()
    h, n = probe_hash(tr)
    assert n == gold["messages"]
    assert f"{h:016x}" == gold["hash"]
    orc = O.Sim(cfg, trace_capacity=1_300_000)
    orc.boot()
    orc.run()
    _assert_same(eng, orc)


@pytest.mark.parametrize("variant", ["lossy", "weights_uniform", "weights_skewed", "runahead",
                                     "bootstrap", "fixed_wide", "floor_rule", "one_host",
                                     "tiny_latency"])
def test_tiny_variants(variant):
    kw = {}
    if variant == "weights_skewed":
        kw["weights"] = np.linspace(0.1, 5.0, 96) ** 2
    cfg = {
        "lossy": lambda: phold.tiny_config(n_hosts=96, loss=0.2),
        "weights_uniform": lambda: phold.tiny_config(n_hosts=96),
        "weights_skewed": lambda: phold.tiny_config(n_hosts=96, **kw),
        "runahead": lambda: phold.tiny_config(n_hosts=96, runahead_ms=7),
        "bootstrap": lambda: dict(phold.tiny_config(n_hosts=96, loss=0.5), bootstrap_end=100_000_000),
        "fixed_wide": lambda: phold.tiny_config(n_hosts=96, window_rule=L.SG_WINDOW_FIXED) | {"fixed_jump": 25 * L.ONE_MS},
        "floor_rule": lambda: phold.tiny_config(n_hosts=96, dst_rule=L.SG_DST_UNIFORM_FLOOR),
        "one_host": lambda: phold.tiny_config(n_hosts=1, V=1, load=3),
        "tiny_latency": lambda: phold.tiny_config(n_hosts=64, min_ms=0.2),
    }[variant]()
    eng, orc = _run_both(cfg, trace=400_000)
    gs = _assert_same(eng, orc)
    assert gs["pops"] > 0
    gt = np.sort(eng.trace(), order=["host", "pos"])
    ot = np.sort(orc.trace(), order=["host", "pos"])
    assert gt.shape == ot.shape
    for f in ("time", "seq", "host", "src", "pos"):
        assert np.array_equal(gt[f], ot[f]), f


def test_c2_shape_parity():
    """configs[1] shape (uniform 50 ms mesh, weights rule) at 10k hosts for 2 s."""
    cfg = phold.c2_config(n_hosts=10_000, end_time_s=2.0)
    eng, orc = _run_both(cfg)
    gs = _assert_same(eng, orc)
    assert gs["pops"] > 10_000 * 16 * 30


def test_c4_shape_prefix_parity():
    """configs[3] shape (log-normal latency, runahead 1 ms) at 100k hosts, 40 rounds."""
    cfg = phold.c4_config(n_hosts=100_000)
    eng, orc = _run_both(cfg, max_rounds=40)
    _assert_same(eng, orc)


def test_lossy_phold_prefix_parity():
    cfg = phold.lossy_config(n_hosts=20_000)
    eng, orc = _run_both(cfg, max_rounds=60)
    gs = _assert_same(eng, orc)
    assert gs["drop_reliability"] > 0


def test_full_size_c4_invariants():
    """1M hosts: size-independent properties — events are conserved (no loss,
    nothing reaches endTime yet), the pending count stays N*load, every host's
    pops equal its event-id counter minus its sends in flight, and the first
    rounds' digests equal the oracle's (checksum of checksums)."""
    cfg = phold.c4_config(n_hosts=1_000_000)
    eng = Engine(cfg)
    eng.boot()
    eng.run(12)
    st = eng.stats()
    assert st["overflow"] == 0
    assert st["pending"] == 1_000_000 * 16 - st["null_dst"]
    assert st["sends"] + st["null_dst"] == st["pops"] - st["boots"] + st["boots"] * 16
    orc = O.Sim(cfg)
    orc.boot()
    orc.run(12)
    g, o = eng.host_state(), orc.host_state()
    assert int(g["digest"].sum(dtype=np.uint64)) == int(o["digest"].sum(dtype=np.uint64))
    assert np.array_equal(g["digest"], o["digest"])


@pytest.mark.parametrize("cap", [1, 128])
def test_queue_capacity_paths(cap):
    """queue_cap sizes the calendar's chunk pool (n_local * queue_cap events plus
    one chunk per ring sub-list and the stashes).  A pool far below the live event count must fail
    loudly (SG_ERR_OVERFLOW), never silently; a large one stays bit-exact."""
    if cap == 1:
        # log-normal delays keep events in many future buckets (with C2's one
        # 50 ms path every new event is due in the next window and k_scatter
        # routes it past the calendar, so that config needs no chunks at all)
        # (the pool also holds one chunk per ring sub-list and the reserving
        # workgroups' stashes, about 12.7k chunks here: 200k hosts x 128 live
        # events need twice that)
        cfg = phold.c4_config(n_hosts=200_000, V=64, end_time_s=0.3, load=128)
        eng = Engine(cfg, queue_cap=cap)
        eng.boot()
        with pytest.raises(L.SgError) as ei:
            eng.run()
        assert ei.value.code == L.SG_ERR_OVERFLOW
        return
    cfg = phold.probe_config(n_hosts=300, jump_ms=10, end_time_s=0.5)
    eng, orc = _run_both(cfg, trace=200_000, queue_cap=cap)
    _assert_same(eng, orc)


def test_c3_shape_bundled_topology():
    """configs[2] shape: hosts attached to the reference's bundled topology
    (country hints on the relays), direct paths of the complete graph."""
    cfg = phold.c3_config(n_relays=400, n_clients=1600, end_time_s=0.4)
    eng, orc = _run_both(cfg)
    gs = _assert_same(eng, orc)
    assert gs["pops"] > 20_000 and gs["drop_reliability"] > 0


def test_incomplete_topology_shortest_paths():
    """An incomplete GraphML graph: shortest paths, paths to self and
    source-wide discovery in the jump table, the same on both sides."""
    import sys
    sys.path.insert(0, os.path.dirname(__file__))
    from test_topology import _graphml, _random_graph
    from shadow_amd import topology as T
    rs = np.random.default_rng(11)
    g = T.Graph(_graphml(30, _random_graph(rs, 30, 0.1), vloss=rs.uniform(0, 0.02, 30)))
    cfg = phold.topology_config(g, 900, load=4, end_time_s=0.5)
    eng, orc = _run_both(cfg)
    _assert_same(eng, orc)


def test_pop_trace_diff_tool():
    """The trace tool on the device and oracle pop traces of the same config."""
    from shadow_amd import trace as T
    cfg = phold.tiny_config(n_hosts=256, V=6, load=4, end_time_s=0.3, loss=0.05)
    eng, orc = _run_both(cfg, trace=1 << 20)
    r = T.diff(eng.trace(), orc.trace())
    assert r["identical"] and r["pops_a"] == eng.stats()["pops"] > 0


@pytest.mark.parametrize("kind", ["lossy", "bootstrap_heavy"])
def test_path_packet_counters(kind):
    """topology_incrementPathPacketCounter (topology.c:2053-2063): kept sends per
    vertex pair, identical to the oracle's, across the inline, phase B and
    same-round paths of k_proc."""
    cfg = {"lossy": lambda: phold.tiny_config(n_hosts=300, V=7, load=4, end_time_s=0.4, loss=0.2),
           "bootstrap_heavy": lambda: dict(phold.tiny_config(n_hosts=200, V=5, load=24, end_time_s=0.3,
                                                             loss=0.3), bootstrap_end=50_000_000)}[kind]()
    eng = Engine(cfg)
    eng.path_counters(True)
    eng.boot()
    eng.run()
    orc = O.Sim(cfg)
    orc.boot()
    orc.run()
    _assert_same(eng, orc)
    g, o = eng.path_counts(), orc.path_counts()
    assert g.sum() > 0 and np.array_equal(g, o)
    st = orc.stats()
    assert int(o.sum()) == st["sends"] - st["drop_reliability"]


def test_path_counters_off_by_default():
    cfg = phold.tiny_config(n_hosts=64)
    eng = Engine(cfg)
    eng.boot()
    eng.run(5)
    assert eng.path_counts().size == 0


@pytest.mark.parametrize("fmt,probe,light,light_q,tri", [(0, False, 2, 1, 1), (1, False, 2, 1, 1),
                                                        (2, True, 2, 1, 1), (2, False, 0, 1, 1),
                                                        (2, False, 2, 99, 1), (2, False, 2, 1, 0),
                                                        (1, False, 2, 1, 0)])
def test_forced_wide_tables(fmt, probe, light, light_q, tri, monkeypatch):
    """configs[3] keeps every packet and has uniform weights, so the engine picks
    the 4-byte delay-only path records and the 2-byte vertex table (the guessed
    host is the drawn one for every x).  Forcing the 16-byte (0) or 8-byte (1)
    path records, or the three-record destination probe, or sending every
    host's sends through phases B and C, or running every light host inline,
    must give the same bits (the switches are read at sg_engine_create).  Its
    paths are symmetric, so the narrow tables hold the lower triangle only;
    tri=0 forces the full V*V tables."""
    monkeypatch.setenv("SG_PAIR_FMT", str(fmt))
    if not tri:
        monkeypatch.setenv("SG_NO_TRI", "1")
    if probe:
        monkeypatch.setenv("SG_NO_EXACT_DST", "1")
    monkeypatch.setenv("SG_LIGHT_MAX", str(light))  # 0: every host's sends through phases B and C
    monkeypatch.setenv("SG_LIGHT_Q", str(light_q))  # 99: every light host inline in phase A
    cfg = phold.c4_config(n_hosts=20_000)
    eng, orc = _run_both(cfg, max_rounds=40)
    _assert_same(eng, orc)


def test_long_paths_use_wide_records():
    """A path delay of 2^32 ns (4.29 s) or more does not fit the narrow records:
    the engine keeps the 16-byte ones and the arithmetic stays 64-bit."""
    lat, el = phold.lognormal_topology(6, 11, median_ms=2000.0, sigma=1.0, min_ms=1.0, edge_loss=0.05)
    lat = lat.reshape(6, 6)
    lat[0, 5] = lat[5, 0] = 6000.0
    cfg = phold.make_config(n_hosts=48, latency_ms=lat, edge_loss=el, load=3, seed=5,
                            end_time_s=30.0, name="long-paths")
    assert int(cfg["delay_ns"].max()) >= 1 << 32
    eng, orc = _run_both(cfg, trace=200_000)
    gs = _assert_same(eng, orc)
    assert gs["pops"] > 0


@pytest.mark.parametrize("grid", [1, 37, 512])
def test_gather_grid(grid, monkeypatch):
    """k_scatter's gather role over SG_GATHER_GRID workgroups: one (every due
    chunk in one workgroup: the two-pass path every round), an odd count, and
    more workgroups than due chunks must all give the same bits."""
    monkeypatch.setenv("SG_GATHER_GRID", str(grid))
    cfg = phold.c4_config(n_hosts=20_000)
    eng, orc = _run_both(cfg, max_rounds=40)
    _assert_same(eng, orc)


@pytest.mark.parametrize("no_rows", [0, 1])
def test_lds_path_rows_switch(no_rows, monkeypatch):
    """Hosts sit in vertex-sorted slots, so a k_proc partition's path records
    are staged in LDS; SG_NO_LDS_ROWS=1 reads them from HBM instead.  Both,
    on a lossy topology (8-byte records) and configs[3]'s (4-byte), must
    give the same bits."""
    if no_rows:
        monkeypatch.setenv("SG_NO_LDS_ROWS", "1")
    for cfg in (phold.lossy_config(n_hosts=30_000, V=64, end_time_s=0.3),
                phold.c4_config(n_hosts=50_000, V=256, end_time_s=0.2)):
        eng, orc = _run_both(cfg, max_rounds=60)
        _assert_same(eng, orc)


@pytest.mark.parametrize("kind,grec", [("lossy", "1"), ("lossless", "1"), ("many_msgs", "1"), ("lossy", "0")])
def test_gossip_record_path(kind, grec, monkeypatch):
    """configs[4]'s gossip body on the record path (phase A records each first
    receipt's forwards, phases B / C resolve them one lane per send, the
    message id riding in the records): lossy links (phase B / C), lossless
    links (the fused pass), more messages than the record path's seen-set
    registers hold (the sequential body instead) and the record path off
    (SG_GREC=0), each against the oracle with the pop traces diffed."""
    monkeypatch.setenv("SG_GREC", grec)
    loss = (0.0, 0.0) if kind == "lossless" else (0.005, 0.05)
    msgs = 200 if kind == "many_msgs" else 40
    # about 2000 hosts x 8 receipts of each message pop: the trace holds them all
    cfg = phold.c5_config(n_hosts=2000, V=16, msgs=msgs, end_time_s=0.6, loss=loss)
    eng, orc = _run_both(cfg, trace=1 << 22)
    _assert_same(eng, orc)
    key = ["host", "pos"]
    assert np.array_equal(np.sort(eng.trace(), order=key), np.sort(orc.trace(), order=key))
    if kind != "lossless":
        assert orc.stats()["drop_reliability"] > 0


@pytest.mark.parametrize("skip", ["1", "0"])
@pytest.mark.parametrize("cfg_kind", ["c2", "nulls"])
def test_flat_skip_ahead_and_null_draws(skip, cfg_kind, monkeypatch):
    """The flat pass skips a multi-event host's earlier draws with the LCG's
    jump-ahead table (SG_SKIP=1) instead of replaying them (0).  A destination
    draw above the last weight threshold selects no host and consumes one draw,
    not two: k_proc marks such a host and replays it in phase A.  configs[1]'s
    shape (every host 16 events a round; the skip path runs where hosts average
    two or more) plain and with the host range cut to 80 % of RAND_MAX (a fifth
    of the draws select no host, so nearly every host takes the fallback), no
    trace (a trace turns the skip off), 12 rounds against the oracle."""
    monkeypatch.setenv("SG_SKIP", skip)
    cfg = phold.c2_config()  # the skip path runs where hosts average two or more due events
    if cfg_kind == "nulls":
        wt = np.asarray(cfg["weight_thresh"])
        cfg["weight_thresh"] = np.minimum(wt, int(0.8 * 2147483647)).astype(wt.dtype)
    eng, orc = _run_both(cfg, max_rounds=12)
    gs = _assert_same(eng, orc)
    if cfg_kind == "nulls":
        assert gs["null_dst"] > 1000, gs["null_dst"]


@pytest.mark.parametrize("skip", ["1", "0"])
@pytest.mark.parametrize("cut", [False, True])
def test_gossip_draws_after_phase_a(skip, cut, monkeypatch):
    """configs[4]'s gossip record path on lossy links with SG_GSKIP=1: phase A
    records each forward as {state, send index} and a pass of one lane per send
    draws it with the jump-ahead table; a draw that selects no host marks its
    host, whose sends one lane redraws in order (real sends first, pads after).
    SG_GSKIP=0 draws in phase A.  The host range cut to 80 % of RAND_MAX makes a
    fifth of the draws select no host, so the redraw runs for most hosts.  No
    trace (a trace turns the table off); host states and counters against the
    oracle."""
    monkeypatch.setenv("SG_GSKIP", skip)
    cfg = phold.c5_config(n_hosts=2000, V=16, msgs=40, end_time_s=0.6)
    if cut:
        wt = np.asarray(cfg["weight_thresh"])
        cfg["weight_thresh"] = np.minimum(wt, int(0.8 * 2147483647)).astype(wt.dtype)
    eng, orc = _run_both(cfg)
    gs = _assert_same(eng, orc)
    assert orc.stats()["drop_reliability"] > 0
    if cut:
        assert gs["null_dst"] > 1000, gs["null_dst"]


@pytest.mark.parametrize("workload", ["gossip", "lossy", "gossip_flat_off"])
def test_send_records_in_hbm(workload, monkeypatch):
    """Send records past k_proc's LDS share live in HBM (non-temporal stores; a
    load there is waited for where it is issued, so the LDS side never waits for
    the wave's stores).  SG_SND_LDS=0 puts every record there: the gossip record
    path with its flat pass (and with it off, phase A recording), and PHOLD on
    lossy links (phases B / C apart), against the oracle."""
    monkeypatch.setenv("SG_SND_LDS", "0")
    if workload == "gossip_flat_off":
        monkeypatch.setenv("SG_GFLAT", "0")
    if workload.startswith("gossip"):
        cfg = phold.c5_config(n_hosts=2000, V=16, msgs=40, end_time_s=0.6)
        eng, orc = _run_both(cfg)
        assert orc.stats()["drop_reliability"] > 0
    else:
        cfg = phold.lossy_config(n_hosts=30_000, V=64, end_time_s=0.3)
        eng, orc = _run_both(cfg, max_rounds=60)
    _assert_same(eng, orc)
