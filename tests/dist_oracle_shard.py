"""TEST INFRASTRUCTURE: an oracle-backed shard with EngineShard's interface, so
the distributed round protocol (shadow_amd.dist) can be exercised on CPU with
gloo.  Never used by the product path."""
import numpy as np
import torch

from oracle import oracle as O
from shadow_amd.dist import owner_bounds


class OracleShard:
    def __init__(self, cfg, rank, world):
        b = owner_bounds(cfg["n_hosts"], world)
        self.bounds = b
        self.world = world
        self.rank = rank
        self.sim = O.Sim(cfg, first_host=b[rank], n_local=b[rank + 1] - b[rank])

    def boot(self):
        self.sim.boot()

    def process(self):
        self.sim.round_process()
        out = self.sim.outbox()
        owner = np.searchsorted(np.array(self.bounds[1:]), out["dst"], side="right")
        counts = np.bincount(owner, minlength=self.world).astype(np.int64)
        cap = max(1, int(counts.max()) if len(counts) else 1)
        send = torch.zeros((self.world, cap, 3), dtype=torch.int64)
        for p in range(self.world):
            ev = out[owner == p]
            if len(ev):
                tri = np.stack([ev["time"].astype(np.int64), ev["seq"].astype(np.int64),
                                ((ev["dst"].astype(np.uint64) << np.uint64(32)) |
                                 ev["src"].astype(np.uint64)).astype(np.int64)], 1)
                send[p, :len(ev)] = torch.from_numpy(tri)
        return send, torch.from_numpy(counts)

    def insert(self, recv, n):
        if n == 0:
            return
        r = recv.numpy().astype(np.uint64)
        ev = np.zeros(n, O.EVENT_DTYPE)
        ev["time"] = r[:, 0]
        ev["seq"] = r[:, 1]
        ev["dst"] = (r[:, 2] >> np.uint64(32)).astype(np.uint32)
        ev["src"] = (r[:, 2] & np.uint64(0xFFFFFFFF)).astype(np.uint32)
        self.sim.ingest(ev)

    def reduce(self):
        v = [self.sim.local_min(), self.sim.local_jmin(), (1 << 64) - 1]
        return torch.tensor([x - (1 << 64) if x >= (1 << 63) else x for x in v], dtype=torch.int64)

    def window(self, red):
        vals = [int(x) & ((1 << 64) - 1) for x in red.tolist()]
        self.sim.window_apply(vals[0], vals[1])

    def done(self):
        return bool(self.sim.stats()["done"])

    def stats(self):
        return self.sim.stats()
