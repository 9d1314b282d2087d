"""TEST INFRASTRUCTURE: an oracle-backed shard with EngineShard's step
interface (pre / post around one all-to-all), so the distributed step protocol
of shadow_amd.dist — fixed-size exchange blocks with headers, drain steps when
an outbox exceeds exchange_cap, the window from the received headers — can be
exercised on CPU with gloo.  Its blocks have the engine's layout
(sg_engine.hip, write_headers / k_proc's outbox copy): HDR = 4 header rows of
RW = 2 int64 words {n, more, MIN, jmin, overflow, round, time base, 0}, then
16-B event rows {time - the sender's window start (40 bits) | destination's
index in the receiving shard << 40, src << 40 | srcHostEventID}, with the
engine's bounds (a time offset below 2^40, a local destination below 2^24).
Received-event insertion and the window from the headers follow the next
k_proc / k_scatter (step_view).  Never used by the product path."""
import numpy as np
import torch

from oracle import oracle as O
from shadow_amd.dist import owner_bounds

HDR = 4   # header rows (sg_engine.hip HDR)
RW = 2    # int64 words per row (sg_engine.hip RW)
H_N, H_MORE, H_MIN, H_JMIN, H_OVF, H_ROUND, H_BASE = range(7)  # header words (enum Hdr)
M64 = (1 << 64) - 1
M40 = (1 << 40) - 1


def _i64(x: int) -> int:
    x &= M64
    return x - (1 << 64) if x >= (1 << 63) else x


class OracleShard:
    row_words = RW

    def __init__(self, cfg, rank, world, exchange_cap=64):
        b = owner_bounds(cfg["n_hosts"], world)
        self.bounds = b
        self.world = world
        self.rank = rank
        self.sim = O.Sim(cfg, first_host=b[rank], n_local=b[rank + 1] - b[rank])
        # the engine's key layout: src << 40 | srcHostEventID << msg_shift | msg
        self.msg_shift = np.uint64(16 if cfg.get("workload", 0) == 1 else 0)
        self.xcap = exchange_cap
        self.rows = HDR + exchange_cap
        self.recv = torch.zeros((world, self.rows, RW), dtype=torch.int64)
        self.phase = 0
        self.outq = [np.zeros((0, 3), np.int64) for _ in range(world)]
        self.sent = [0] * world
        self.base = 0
        self.loc_min = (1 << 64) - 2
        self.loc_jmin = M64
        self.steps = 0
        self.peak = 0
        # the EngineShard surface dist.bench uses
        self.dev = None
        self.comm = None

    def boot(self):
        self.sim.boot()

    def _done(self):
        return bool(self.sim.stats()["done"])

    def pre(self) -> torch.Tensor:
        send = torch.zeros((self.world, self.rows, RW), dtype=torch.int64)
        if self._done():
            return send
        st = self.sim.stats()
        base = st["window_start"]  # H_BASE: the rows' time base (the step's window start)
        if self.phase == 0:
            self.sim.round_process()
            out = self.sim.outbox()
            owner = np.searchsorted(np.array(self.bounds[1:]), out["dst"], side="right")
            for p in range(self.world):
                ev = out[owner == p] if p != self.rank else out[:0]
                if len(ev):
                    rel = ev["time"].astype(np.uint64) - np.uint64(base)
                    dl = ev["dst"].astype(np.uint64) - np.uint64(self.bounds[p])
                    assert int(rel.max()) < (1 << 40), "time offset beyond 2^40 ns of the window start"
                    assert int(dl.max()) < (1 << 24), "receiving-shard index beyond 24 bits"
                    key = (ev["src"].astype(np.uint64) << np.uint64(40)) | \
                          (ev["seq"].astype(np.uint64) << self.msg_shift) | ev["msg"].astype(np.uint64)
                    self.outq[p] = np.stack([(rel | (dl << np.uint64(40))).astype(np.int64),
                                             key.astype(np.int64)], 1)
                else:
                    self.outq[p] = np.zeros((0, RW), np.int64)
            self.sent = [0] * self.world
            self.peak = max([self.peak] + [len(self.outq[p]) for p in range(self.world) if p != self.rank])
            m = self.sim.local_min()
            if len(out):
                m = min(m, int(out["time"].min()))
            self.loc_min = m
            self.loc_jmin = self.sim.local_jmin()
            self.base = base
        more = any(len(self.outq[q]) - self.sent[q] > self.xcap for q in range(self.world))
        rounds = self.sim.stats()["rounds"]
        for p in range(self.world):
            n = min(self.xcap, len(self.outq[p]) - self.sent[p])
            h = send[p, :HDR].view(-1)
            h[H_N], h[H_MORE], h[H_MIN] = n, int(more), _i64(self.loc_min)
            h[H_JMIN], h[H_OVF], h[H_ROUND], h[H_BASE] = _i64(self.loc_jmin), 0, rounds, _i64(self.base)
            if n:
                send[p, HDR:HDR + n] = torch.from_numpy(self.outq[p][self.sent[p]:self.sent[p] + n])
        return send

    def post(self):
        if self._done():
            return
        r = self.recv.numpy()
        m = j = M64
        more = False
        for p in range(self.world):
            h = r[p, :HDR].reshape(-1)
            more |= bool(h[H_MORE])
            m = min(m, int(h[H_MIN]) & M64)
            j = min(j, int(h[H_JMIN]) & M64)
            assert int(h[H_ROUND]) == self.sim.stats()["rounds"], "shards out of step"
            n = int(h[H_N])
            if p == self.rank or n == 0:
                continue
            rows = r[p, HDR:HDR + n].astype(np.uint64)
            ev = np.zeros(n, O.EVENT_DTYPE)
            ev["time"] = np.uint64(int(h[H_BASE]) & M64) + (rows[:, 0] & np.uint64(M40))
            low = rows[:, 1] & np.uint64(M40)
            ev["seq"] = low >> self.msg_shift
            ev["msg"] = low & ((np.uint64(1) << self.msg_shift) - np.uint64(1))
            ev["src"] = (rows[:, 1] >> np.uint64(40)).astype(np.uint32)
            ev["dst"] = ((rows[:, 0] >> np.uint64(40)) + np.uint64(self.bounds[self.rank])).astype(np.uint32)
            self.sim.ingest(ev)
        for q in range(self.world):
            self.sent[q] += min(self.xcap, len(self.outq[q]) - self.sent[q])
        self.steps += 1
        if more:
            self.phase = 1
            return
        self.phase = 0
        self.sim.window_apply(m, j)

    def done(self):
        return self._done()

    def stats(self):
        st = self.sim.stats()
        st["exchange_steps"] = self.steps
        st["phase"] = self.phase
        st.setdefault("overflow", 0)
        return st

    # ---- the rest of EngineShard's surface (dist.bench)
    def exchange_peak(self, reset=False):
        v = self.peak
        if reset:
            self.peak = 0
        return v

    def set_exchange_cap(self, cap):
        self.xcap = cap
        self.rows = HDR + cap
        self.recv = torch.zeros((self.world, self.rows, RW), dtype=torch.int64)

    def sync(self):
        pass

    def close_native(self):
        pass

    def fingerprint(self):
        from shadow_amd.trace import state_fingerprint
        hs = self.sim.host_state()
        return state_fingerprint(self.bounds[self.rank], hs["digest"], hs["pops"], hs["rng"], hs["ev"])
