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


def _run_shards(cfg, world, xcap, trace=0):
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


@pytest.mark.parametrize("graph", [3, 8])
def test_graph_rounds_match_oracle(graph):
    """Round mode replayed from captured hipGraphs (sg_engine_run and
    sg_engine_enqueue_rounds), including a partial last batch."""
    from shadow_amd.engine import Engine
    cfg = phold.c4_config(n_hosts=40_000, V=64, end_time_s=0.2)
    eng = Engine(cfg, device=0)
    eng.boot()
    eng.set_graph(graph)
    eng.enqueue_rounds(2 * graph + 1)
    eng.run(batch=graph)
    ref = O.Sim(cfg)
    ref.boot()
    ref.run()
    g, o = eng.host_state(), ref.host_state()
    for k in ("digest", "pops", "rng", "ev"):
        assert np.array_equal(g[k], o[k]), k
    assert eng.stats()["rounds"] == ref.stats()["rounds"]
