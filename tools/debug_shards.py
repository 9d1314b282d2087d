"""Debug: in-process shards vs oracle — window sequences and first diverging host."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
from shadow_amd import phold
from shadow_amd.dist import EngineShard
from oracle import oracle as O

def flip(t):
    return torch.bitwise_xor(t, torch.tensor(-(1 << 63), dtype=torch.int64, device=t.device))

world = int(sys.argv[1]) if len(sys.argv) > 1 else 4
cfg = phold.c4_config(n_hosts=40_000, V=64, end_time_s=0.2)
shards = [EngineShard(cfg, r, world, 0) for r in range(world)]
for s in shards:
    s.eng.close()
from shadow_amd.engine import Engine
stream = torch.cuda.Stream()
for r, s in enumerate(shards):
    s.eng = Engine(cfg, device=0, shard_index=r, shard_count=world, exchange_cap=s.cap,
                   trace_capacity=1 << 22, stream=stream.cuda_stream)
    s.stream = stream
    s.boot()
torch.cuda.set_stream(stream)
rounds = 0
while rounds < 400:
    sends = [s.process() for s in shards]
    torch.cuda.synchronize()
    for r, s in enumerate(shards):
        parts = [sends[p][0][r, :int(sends[p][1][r])] for p in range(world)]
        recv = torch.cat(parts, 0).contiguous()
        s.insert(recv, recv.shape[0])
    reds = [flip(s.reduce().clone()) for s in shards]
    torch.cuda.synchronize()
    g = flip(torch.stack(reds).min(0).values)
    for s in shards:
        s.window(g)
    torch.cuda.synchronize()
    rounds += 1
    if shards[0].done():
        break
ref = O.Sim(cfg, trace_capacity=1 << 22)
ref.boot(); ref.run()
ow = ref.windows()
for r, s in enumerate(shards):
    w = s.eng.windows()
    n = min(len(w), len(ow))
    bad = np.nonzero((w[:n] != ow[:n]).any(1))[0]
    print("shard", r, "windows", len(w), "oracle", len(ow), "first diff", bad[:3], w[bad[:1]], ow[bad[:1]], s.stats()["overflow"])
hs = [s.eng.host_state() for s in shards]
dg = np.concatenate([h["digest"] for h in hs]); od = ref.host_state()["digest"]
bad = np.nonzero(dg != od)[0]
print("bad hosts", len(bad), bad[:10])
if len(bad):
    gt = np.concatenate([s.eng.trace() for s in shards]); gt = np.sort(gt, order=["host", "pos"])
    ot = np.sort(ref.trace(), order=["host", "pos"])
    h0 = bad[0]
    a = gt[gt["host"] == h0]; b = ot[ot["host"] == h0]
    print("host", h0, len(a), len(b))
    for i in range(min(len(a), len(b))):
        if (a[i]["time"], a[i]["src"], a[i]["seq"]) != (b[i]["time"], b[i]["src"], b[i]["seq"]):
            print("pos", i, "gpu", a[max(0,i-1):i+2], "orc", b[max(0,i-1):i+2]); break
