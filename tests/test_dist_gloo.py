"""CPU, world size 2, 3, 4 and 8 over gloo (PHOLD and the gossip body): the distributed step protocol of
shadow_amd.dist (one all-to-all of fixed-size blocks per step, the window from
the block headers, drain steps when an outbox exceeds the block) reproduces
the unsharded simulation exactly (per-host digests, pops, RNG states, event
counters, global counters)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from shadow_amd import phold


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, cfg, xcap, q, stop_round=0):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from tests.dist_oracle_shard import OracleShard
    from shadow_amd import dist as D
    sh = OracleShard(cfg, rank, world, exchange_cap=xcap)
    sh.boot()
    if stop_round:
        # the bench's path: a batch of steps that may end on a drain step, then
        # finish_round to the next round boundary on every rank
        D.run_until_round(sh, world, stop_round, check_every=3)
        D.finish_round(sh, world)
        rounds = sh.stats()["rounds"]
    else:
        rounds = D.run(sh, world, check_every=4)
    st = sh.sim.host_state()
    q.put((rank, rounds, sh.stats(), {k: v.copy() for k, v in st.items()}))
    dist.barrier()
    dist.destroy_process_group()


def _run(cfg, world, xcap, stop_round=0):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, cfg, xcap, q, stop_round))
          for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    return sorted(res, key=lambda x: x[0])


@pytest.mark.parametrize("world,kind,xcap", [(2, "tiny", 64), (3, "lossy", 16), (2, "probe10", 4096),
                                             (2, "tiny", 3), (8, "tiny", 8), (4, "gossip", 16),
                                             (8, "gossip", 64)])
def test_sharded_protocol_matches_unsharded(world, kind, xcap):
    from oracle import oracle as O
    cfg = {"tiny": lambda: phold.tiny_config(n_hosts=200, V=6, load=4, end_time_s=0.4),
           "lossy": lambda: phold.tiny_config(n_hosts=151, V=5, load=3, loss=0.3, end_time_s=0.3),
           "probe10": lambda: phold.probe_config(n_hosts=120, jump_ms=10, end_time_s=0.3),
           "gossip": lambda: phold.c5_config(n_hosts=400, V=6, msgs=12, fanout=4, end_time_s=1.0)}[kind]()
    res = _run(cfg, world, xcap)
    ref = O.Sim(cfg)
    ref.boot()
    ref.run()
    rs = ref.host_state()
    for k in ("digest", "pops", "rng", "ev"):
        got = np.concatenate([r[3][k] for r in res])
        assert np.array_equal(got, rs[k]), k
    tot = {k: sum(r[2][k] for r in res) for k in ("pops", "sends", "drop_reliability",
                                                  "drop_endtime", "bumped", "same_round")}
    want = ref.stats()
    for k, v in tot.items():
        assert v == want[k], (k, v, want[k])
    for r in res:  # every rank ran the same windows and steps, and ended in the same state
        assert r[2]["rounds"] == want["rounds"]
        assert r[2]["window_start"] == want["window_start"]
        assert r[2]["exchange_steps"] == res[0][2]["exchange_steps"]
    if xcap <= 16:  # small blocks: the boot round's outbox must have drained over extra steps
        assert res[0][2]["exchange_steps"] > want["rounds"]


def test_finish_round_stops_at_a_round_boundary():
    """dist.run_until_round + dist.finish_round (the bench's parity point) end
    every rank at the same round boundary, after a batch that can end inside a
    drain step (tiny blocks), with the state of the unsharded run at that round."""
    from oracle import oracle as O
    cfg = phold.tiny_config(n_hosts=200, V=6, load=4, end_time_s=0.4)
    res = _run(cfg, 2, 3, stop_round=7)
    r0 = res[0][1]
    assert r0 >= 7 and all(r[1] == r0 for r in res)
    assert all(r[2]["phase"] == 0 for r in res)
    ref = O.Sim(cfg)
    ref.boot()
    ref.run(r0)
    rs = ref.host_state()
    for k in ("digest", "pops", "rng", "ev"):
        assert np.array_equal(np.concatenate([r[3][k] for r in res]), rs[k]), k


def _bench_worker(rank, world, port, q):
    import argparse
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from tests.dist_oracle_shard import OracleShard
    from shadow_amd import dist as D
    args = argparse.Namespace(gpus=world, same_device=True, dist_backend="gloo", hosts=3000,
                              py_steps=True, graph=0, warmup=4, steps=12, kernel_rounds=4)
    try:
        res = D.bench(args, make_shard=lambda cfg, r, w, dev: OracleShard(cfg, r, w, exchange_cap=64))
        q.put((rank, res, None))
    except BaseException as exc:  # noqa: BLE001
        import traceback
        q.put((rank, None, traceback.format_exc()))


def test_dist_bench_runs_on_cpu():
    """dist.bench itself (the N > 1 bench path: warmup, exchange-block sizing from
    the peak, the timed steps, finish_round, the summed fingerprint) over gloo
    with oracle-backed shards; the end-state fingerprint it reports equals the
    unsharded oracle's at the same round."""
    from oracle import oracle as O
    from shadow_amd.trace import state_fingerprint
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_bench_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = sorted([q.get(timeout=300) for _ in range(2)], key=lambda x: x[0])
    for p in ps:
        p.join(60)
    assert not out[0][2] and not out[1][2], out[0][2] or out[1][2]
    res = out[0][1]
    assert out[1][1] is None and res["n_gpus"] == 2 and res["value"] > 0
    assert res["config"]["rounds_timed"] >= 1
    ref = O.Sim(phold.c4_config(n_hosts=3000))
    ref.boot()
    ref.run(res["_end_round"])
    hs = ref.host_state()
    assert res["_fingerprint"] == state_fingerprint(0, hs["digest"], hs["pops"], hs["rng"], hs["ev"])
