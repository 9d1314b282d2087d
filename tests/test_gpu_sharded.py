"""GPU: the sharded engine path (k_proc writing the outbox and exchange
blocks and queueing the previous step's received events, k_scatter routing the
received events due in the new window: one
all-to-all of fixed-size blocks per step, the window from the block headers,
drain steps) with several shards on one device.  The
all-to-all is done in-process with block copies on the shards' common stream,
exactly as shadow_amd.dist does over RCCL; results must equal the unsharded
oracle."""
import numpy as np
import pytest
import torch

from shadow_amd import phold
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _run_shards(cfg, world, xcap, trace=0, between=None):
    """between(step, shards): called after each step's post (on the stream)."""
    from shadow_amd.dist import EngineShard
    stream = torch.cuda.Stream()
    shards = [EngineShard(cfg, r, world, 0, exchange_cap=xcap, stream=stream, trace_capacity=trace)
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
            if between is not None:
                between(steps, shards)
            if steps % 8 == 0 and shards[0].done():
                break
            assert steps < 200_000
    stream.synchronize()
    return shards, steps


def _check(cfg, shards):
    ref = O.Sim(cfg)
    ref.boot()
    ref.run()
    rs = ref.host_state()
    st = [s.stats() for s in shards]
    assert all(x["overflow"] == 0 for x in st), [hex(x["overflow"]) for x in st]
    hs = [s.eng.host_state() for s in shards]
    for k in ("digest", "pops", "rng", "ev"):
        assert np.array_equal(np.concatenate([h[k] for h in hs]), rs[k]), k
    want = ref.stats()
    for k in ("pops", "sends", "drop_reliability", "drop_endtime", "bumped", "same_round"):
        assert sum(x[k] for x in st) == want[k], k
    for x in st:
        assert x["rounds"] == want["rounds"], (x["rounds"], want["rounds"])
        assert (x["window_start"], x["window_end"]) == (want["window_start"], want["window_end"])
        assert x["exchange_steps"] == st[0]["exchange_steps"]
    return st, want


@pytest.mark.parametrize("world,kind,xcap", [(1, "tiny", 4096), (1, "c4small", None),
                                             (2, "tiny", 4096), (3, "probe10", 4096),
                                             (4, "c4small", None), (2, "tiny", 7),
                                             (3, "lossy", 50)])
def test_inprocess_shards_match_oracle(world, kind, xcap):
    cfg = {"tiny": lambda: phold.tiny_config(n_hosts=500, V=6, load=4, end_time_s=0.4, loss=0.1),
           "lossy": lambda: phold.tiny_config(n_hosts=301, V=5, load=3, loss=0.3, end_time_s=0.3),
           "probe10": lambda: phold.probe_config(n_hosts=400, jump_ms=10, end_time_s=0.5),
           "c4small": lambda: phold.c4_config(n_hosts=40_000, V=64, end_time_s=0.2)}[kind]()
    shards, steps = _run_shards(cfg, world, xcap)
    st, want = _check(cfg, shards)
    if xcap is not None and xcap < 64:  # the boot outboxes drained over extra steps
        assert st[0]["exchange_steps"] > want["rounds"]


@pytest.mark.parametrize("gspec", ["1", "0", "2"])
def test_sharded_gspec_modes_match_oracle(gspec, monkeypatch):
    """The step path's gather with the GSpec guess on (hits in steady rounds),
    off (SG_GSPEC=0: the list path every round) and deliberately wrong
    (SG_GSPEC=2: the guess names the bucket after the right one, and the
    gather must reject it and take the list path), 4 shards, against the
    oracle.  (Round 5's split step, k_spec beside the exchange, was removed
    in round 6: profiles/r05/split.)"""
    monkeypatch.setenv("SG_GSPEC", gspec)  # read when the engines are created
    # V = 1024 as in configs[3]: the discovered minimum is 1 ms, so steady
    # windows are one whole bucket (V = 64 leaves 2-3 ms windows: no guess)
    cfg = phold.c4_config(n_hosts=60_000, end_time_s=0.15)
    shards, _ = _run_shards(cfg, 4, None)
    _check(cfg, shards)
    g = [s.eng.gather_paths() for s in shards]
    if gspec == "1":
        assert all(x["guessed"] > 0 for x in g), g
    else:
        assert all(x["guessed"] == 0 and x["listed"] > 0 for x in g), g


def test_sharded_windows_and_trace_match_oracle():
    cfg = phold.probe_config(n_hosts=300, jump_ms=10, end_time_s=0.3)
    shards, _ = _run_shards(cfg, 3, 16, trace=1 << 20)
    ref = O.Sim(cfg, trace_capacity=1 << 21)
    ref.boot()
    ref.run()
    w = ref.windows()
    for s in shards:
        assert np.array_equal(s.eng.windows(), w)
    tr = np.concatenate([s.eng.trace() for s in shards])
    rt = ref.trace()
    key = ["host", "pos"]
    assert np.array_equal(np.sort(tr, order=key), np.sort(rt, order=key))


@pytest.mark.parametrize("xcap", [4096, 7])
@pytest.mark.parametrize("fuse", ["1", "0"])
@pytest.mark.parametrize("fence", ["", "1"])
def test_xlink_steps_world1_match_oracle(xcap, fuse, fence, monkeypatch):
    """sg_engine_run_steps_xlink at world 1: every block goes through k_xpush
    into this shard's own exchange region (uncached memory, parity buffers,
    arrival counters) and k_xwait, after a pattern self-test; a 7-row cap
    (no event crosses a shard at world 1: only the block size changes); with and without the system-scope release before each
    arrival (SG_XFENCE=1; the default fences only across devices).  SG_XFUSE=1 (the default): k_proc stores the blocks
    into the region itself and its last workgroup signals; 0: k_xpush copies
    them after it.  Half way the link is closed (the last received blocks are
    copied back into the engine) and the run finishes on in-process block
    copies."""
    from shadow_amd.dist import EngineShard
    monkeypatch.setenv("SG_XFUSE", fuse)  # read by sg_xlink_create
    monkeypatch.setenv("SG_XFENCE", fence)  # "": the default (no peer on another device: unfenced)
    from shadow_amd.engine import XLink
    cfg = phold.tiny_config(n_hosts=500, V=6, load=4, end_time_s=0.4, loss=0.1)
    sh = EngineShard(cfg, 0, 1, 0, exchange_cap=xcap)
    sh.boot()
    xl = XLink(sh.eng)
    xl.attach(xl.handle())  # world 1: only this shard's own region, no IPC mapping
    assert xl.selftest(6) == 0
    sh.xl = xl
    n = 0
    while not sh.done() and n < 24:
        sh.run_native(8)
        n += 8
    assert not xl.timed_out()
    xl.close()
    sh.xl = None
    with torch.cuda.stream(sh.stream):
        while not sh.done():
            send = sh.pre()
            sh.recv.copy_(send)
            sh.post()
            n += 1
            assert n < 100_000
    sh.sync()
    _check(cfg, [sh])


@pytest.mark.parametrize("fence", ["", "1"])
def test_xlink_selftest_runs_the_fused_protocol(fence, monkeypatch):
    """The self-test that decides between the xGMI link and RCCL exercises the
    path real steps take (SG_XFUSE=1, the default): k_xfused's 128 workgroups
    store into the region, release, take a ticket, and the last one writes
    the headers and arrives; 64 exchanges (every fourth a full block) check
    clean, fenced and unfenced, and the link reports what it ran."""
    from shadow_amd.dist import EngineShard
    from shadow_amd.engine import XLink
    monkeypatch.setenv("SG_XFENCE", fence)
    cfg = phold.tiny_config(n_hosts=500, V=6, load=4, end_time_s=0.4, loss=0.1)
    sh = EngineShard(cfg, 0, 1, 0, exchange_cap=4096)
    sh.boot()
    xl = XLink(sh.eng)
    xl.attach(xl.handle())
    assert xl.selftest(64) == 0
    info = xl.info()
    assert info["fused"] == 1 and info["selftest_fused"] == 1 and info["selftest_steps"] == 64
    assert info["selftest_bad"] == 0 and info["steps"] == 64 and info["shared_device"] == 0
    assert info["fenced"] == (1 if fence else 0)
    xl.close()


@pytest.mark.timeout(60)
def test_xlink_withheld_arrival_fails_fast():
    """A sender that never arrives (sg_xlink_debug_withhold: the next fused
    step skips its arrival) must fail the run fast: the wait gives up once
    (5 s), every later wait of the link returns at once, the run stops
    (OV_XCHG) and the host's check raises naming the missing shard — within
    10 s for 40 steps, where a wait per step would take 200 s.  World 1: the
    wait is k_scatter's in-kernel one, the one ranks on different GPUs take."""
    import time
    from shadow_amd.dist import EngineShard
    from shadow_amd.engine import XLink
    cfg = phold.tiny_config(n_hosts=500, V=6, load=4, end_time_s=0.4, loss=0.1)
    sh = EngineShard(cfg, 0, 1, 0, exchange_cap=4096)
    sh.boot()
    xl = XLink(sh.eng)
    xl.attach(xl.handle())
    assert xl.selftest(4) == 0
    sh.xl = xl
    sh.run_native(2)
    xl.debug_withhold(1, 0)
    t0 = time.perf_counter()
    with pytest.raises(RuntimeError, match=r"no arrival from shard\(s\) \[0\]"):
        sh.run_native(40)
    dt = time.perf_counter() - t0
    assert dt < 10.0, dt
    st = sh.stats()
    assert st["overflow"] & 8 and st["done"], st  # OV_XCHG: the run stopped
    sh.xl = None
    xl.close()


@pytest.mark.parametrize("graph", [0, 4])
def test_native_rccl_steps_world1_match_oracle(graph):
    """sg_engine_run_steps: step_send, RCCL all-to-all (a world-1 communicator of
    libshadowgpu's own) and step_recv issued from C, optionally replayed from
    captured hipGraphs; a small exchange_cap forces drain steps."""
    from shadow_amd.dist import EngineShard
    from shadow_amd.engine import Comm
    cfg = phold.tiny_config(n_hosts=500, V=6, load=4, end_time_s=0.4, loss=0.1)
    sh = EngineShard(cfg, 0, 1, 0, exchange_cap=4096)
    sh.comm = Comm(Comm.unique_id(), 0, 1, 0)
    sh.eng.set_graph(graph)
    sh.boot()
    n = 0
    while not sh.done():
        sh.run_native(8)
        n += 8
        assert n < 100_000
    sh.sync()
    _check(cfg, [sh])
    sh.close_native()


@pytest.mark.parametrize("graph,prepare", [(3, False), (8, False), (8, True)])
def test_graph_rounds_match_oracle(graph, prepare):
    """Round mode replayed from captured hipGraphs (sg_engine_run and
    sg_engine_enqueue_rounds), including a partial last batch; prepare: the
    graph captured ahead by sg_engine_graph_prepare, which must run nothing."""
    from shadow_amd.engine import Engine
    cfg = phold.c4_config(n_hosts=40_000, V=64, end_time_s=0.2)
    eng = Engine(cfg, device=0)
    eng.boot()
    eng.set_graph(graph)
    if prepare:
        r0 = eng.stats()["rounds"]
        eng.prepare_graph()
        eng.prepare_graph()  # the same key: kept
        assert eng.stats()["rounds"] == r0
    eng.enqueue_rounds(2 * graph + 1)
    eng.run(batch=graph)
    ref = O.Sim(cfg)
    ref.boot()
    ref.run()
    g, o = eng.host_state(), ref.host_state()
    for k in ("digest", "pops", "rng", "ev"):
        assert np.array_equal(g[k], o[k]), k
    assert eng.stats()["rounds"] == ref.stats()["rounds"]


def test_graph_prepare_runs_nothing_when_eager():
    """sg_engine_graph_prepare under a setting that makes enqueue_batch launch
    eagerly (kernel timing on): it must neither capture nor run rounds, so the
    round count and the host state stay where they were."""
    from shadow_amd.engine import Engine
    cfg = phold.c4_config(n_hosts=40_000, V=64, end_time_s=0.2)
    eng = Engine(cfg, device=0)
    eng.boot()
    eng.run(3, batch=3)
    eng.set_graph(8)
    eng.set_timing(True)
    r0 = eng.stats()["rounds"]
    d0 = eng.host_state()["digest"].copy()
    eng.prepare_graph()
    assert eng.stats()["rounds"] == r0
    assert np.array_equal(eng.host_state()["digest"], d0)
    eng.set_timing(False)
    eng.set_graph(0)


POISON = -0x0123456789ABCDF  # not a valid event row or header


def test_exchange_cap_change_keeps_received_blocks():
    """sg_engine_set_exchange_cap between steps while the last received blocks
    are still unconsumed (the next k_proc stages the ones k_scatter did not
    route): the caller reallocates its buffers, and the new receive buffer is
    poisoned, so a k_proc that read it instead of the engine's copy would
    diverge (the round-3 mismatch, gpurun_out/ab/sharded.log).  Changes land on
    process steps and on drain steps, shrinking and growing the blocks."""
    cfg = phold.tiny_config(n_hosts=600, V=6, load=6, end_time_s=0.4, loss=0.1)
    plan = {3: 4096, 5: 9, 9: 40, 14: 4096, 20: 13}
    seen = {"drain": 0, "process": 0}

    def between(step, shards):
        cap = plan.get(step)
        if cap is None and step > 20 and step % 7 == 0:
            cap = 13 if shards[0].eng.exchange_rows() > 100 else 4096
        if cap is None:
            return
        st = shards[0].stats()
        seen["drain" if st["phase"] else "process"] += 1
        for sh in shards:
            sh.set_exchange_cap(cap)
            sh.recv.fill_(POISON)
            sh.send.fill_(POISON)

    shards, _ = _run_shards(cfg, 3, 4096, between=between)
    st, want = _check(cfg, shards)
    assert st[0]["exchange_steps"] > want["rounds"]  # small caps drained over extra steps
    assert seen["drain"] >= 1 and seen["process"] >= 1, seen


def test_native_exchange_cap_change_world1():
    """The native step loop (world-1 RCCL communicator) with exchange_cap changed
    between batches of steps: buffers reallocated and poisoned, graphs rebuilt."""
    from shadow_amd.dist import EngineShard
    from shadow_amd.engine import Comm
    cfg = phold.tiny_config(n_hosts=500, V=6, load=4, end_time_s=0.4, loss=0.1)
    sh = EngineShard(cfg, 0, 1, 0, exchange_cap=4096)
    sh.comm = Comm(Comm.unique_id(), 0, 1, 0)
    sh.eng.set_graph(4)
    sh.boot()
    n, caps = 0, [256, 4096, 512, 1024]
    while not sh.done():
        sh.run_native(8)
        n += 8
        sh.set_exchange_cap(caps[(n // 8) % len(caps)])
        with sh.stream_ctx():  # ordered before the next steps on the engine stream
            sh.recv.fill_(POISON)
            sh.send.fill_(POISON)
        assert n < 100_000
    sh.sync()
    _check(cfg, [sh])
    sh.close_native()
