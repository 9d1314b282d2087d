"""GPU: the sharded engine path (k_peer_scan, k_pack, k_insert_recv, split
reduce/window) with several shards on one device, exchanging in-process exactly
as shadow_amd.dist does over RCCL; must equal the unsharded oracle."""
import numpy as np
import pytest
import torch

from shadow_amd import phold
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _flip(t):
    return torch.bitwise_xor(t, torch.tensor(-(1 << 63), dtype=torch.int64, device=t.device))


@pytest.mark.parametrize("world,kind", [(2, "tiny"), (3, "probe10"), (4, "c4small")])
def test_inprocess_shards_match_oracle(world, kind):
    from shadow_amd.dist import EngineShard
    from shadow_amd.engine import Engine
    cfg = {"tiny": lambda: phold.tiny_config(n_hosts=500, V=6, load=4, end_time_s=0.4, loss=0.1),
           "probe10": lambda: phold.probe_config(n_hosts=400, jump_ms=10, end_time_s=0.5),
           "c4small": lambda: phold.c4_config(n_hosts=40_000, V=64, end_time_s=0.2)}[kind]()
    shards = [EngineShard(cfg, r, world, 0) for r in range(world)]
    stream = torch.cuda.Stream()
    for s in shards:  # one stream for everything, as one rank's round would be
        s.eng.close()
        s.stream = stream
        s.eng = Engine(cfg, device=0, shard_index=s.eng_args[0], shard_count=world,
                       exchange_cap=s.cap, stream=stream.cuda_stream)
        s.boot()
    ctx = torch.cuda.stream(stream)
    ctx.__enter__()
    rounds = 0
    while True:
        sends = [s.process() for s in shards]
        torch.cuda.synchronize()
        for r, s in enumerate(shards):
            parts = [sends[p][0][r, :int(sends[p][1][r])] for p in range(world)]
            recv = torch.cat(parts, 0).contiguous()
            s.insert(recv, recv.shape[0])
        reds = [_flip(s.reduce().clone()) for s in shards]
        torch.cuda.synchronize()
        g = _flip(torch.stack(reds).min(0).values)
        for s in shards:
            s.window(g)
        torch.cuda.synchronize()
        rounds += 1
        if rounds % 8 == 0 and shards[0].done():
            break
        assert rounds < 100_000
    ctx.__exit__(None, None, None)
    ref = O.Sim(cfg)
    ref.boot()
    ref.run()
    rs = ref.host_state()
    hs = [s.eng.host_state() for s in shards]
    for k in ("digest", "pops", "rng", "ev"):
        assert np.array_equal(np.concatenate([h[k] for h in hs]), rs[k]), k
    st = [s.stats() for s in shards]
    want = ref.stats()
    assert all(x["overflow"] == 0 for x in st), [hex(x["overflow"]) for x in st]
    for k in ("pops", "sends", "drop_reliability", "drop_endtime", "bumped", "same_round"):
        assert sum(x[k] for x in st) == want[k], k
    assert all(x["rounds"] == want["rounds"] for x in st), ([x["rounds"] for x in st], want["rounds"], [(x["window_start"], x["window_end"], x["done"]) for x in st], (want["window_start"], want["window_end"]))
