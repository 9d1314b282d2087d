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


def _worker(rank, world, port, cfg, xcap, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from tests.dist_oracle_shard import OracleShard
    from shadow_amd import dist as D
    sh = OracleShard(cfg, rank, world, exchange_cap=xcap)
    sh.boot()
    rounds = D.run(sh, world, check_every=4)
    st = sh.sim.host_state()
    q.put((rank, rounds, sh.stats(), {k: v.copy() for k, v in st.items()}))
    dist.barrier()
    dist.destroy_process_group()


def _run(cfg, world, xcap):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, cfg, xcap, q)) for r in range(world)]
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
