"""TEST INFRASTRUCTURE — a small PHOLD run built on the reference's own compiled
code where it compiles here (oracle/_ref/libshdref.so: utility/random.c and
utility/priority_queue.c, unmodified; `make -C oracle ref`).

What is the reference's own code in this run:
  * every random draw: random_new / random_rand / random_nextDouble /
    random_nextUInt (random.c:20-51) over glibc rand_r, including the seed
    chain master.c:95 -> master.c:417 -> slave.c:182 -> slave.c:198 ->
    slave.c:301 and the attachment draw (topology.c:2327-2333);
  * every per-host event queue: priorityqueue_new / push / peek / pop
    (priority_queue.c:37-175), the binary heap with its GHashTable index,
    ordered by a restatement of event_compare (event.c:110-153; host_compare
    orders hosts by GQuark = registration index, host.c:439-445).

What is restated here (in Python, independently of oracle/orc.c and of the
product's integer tables): the host_single round loop (host_single.c:167-305),
scheduler_push's endTime drop (scheduler.c:339-357), the PHOLD body with the
reference's floating-point rules — destination by cumulative normalised
weights `cumulative >= random()/RAND_MAX` (test_phold.c:107-110, 160-178),
keep iff `chance <= reliability` (worker.c:268-273), `ceil(latency * 1e6)`
delays (worker.c:275-277) — and the window (master.c:133-159, 450-480).

Only tests use it, to pin the oracle (and the product's integer threshold
tables, which it never uses) against reference code.
"""
from __future__ import annotations

import ctypes as C
import ctypes.util
import math
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
REF_LIB = os.path.join(_HERE, "_ref", "libshdref.so")
RAND_MAX = 2147483647
ONE_MS = 1_000_000
SIMTIME_MAX = (1 << 64) - 2
_lib = None


def available() -> bool:
    return os.path.exists(REF_LIB)


def lib():
    global _lib
    if _lib is None:
        L = C.CDLL(REF_LIB)
        L.random_new.restype = C.c_void_p
        L.random_new.argtypes = [C.c_uint]
        L.random_free.argtypes = [C.c_void_p]
        L.random_rand.restype = C.c_int
        L.random_rand.argtypes = [C.c_void_p]
        L.random_nextDouble.restype = C.c_double
        L.random_nextDouble.argtypes = [C.c_void_p]
        L.random_nextUInt.restype = C.c_uint
        L.random_nextUInt.argtypes = [C.c_void_p]
        L.priorityqueue_new.restype = C.c_void_p
        L.priorityqueue_new.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        L.priorityqueue_free.argtypes = [C.c_void_p]
        L.priorityqueue_push.restype = C.c_int
        L.priorityqueue_push.argtypes = [C.c_void_p, C.c_void_p]
        L.priorityqueue_peek.restype = C.c_void_p
        L.priorityqueue_peek.argtypes = [C.c_void_p]
        L.priorityqueue_pop.restype = C.c_void_p
        L.priorityqueue_pop.argtypes = [C.c_void_p]
        L.priorityqueue_getLength.restype = C.c_size_t
        L.priorityqueue_getLength.argtypes = [C.c_void_p]
        _lib = L
    return _lib


_libm = C.CDLL(ctypes.util.find_library("m"))
_libm.round.restype = C.c_double
_libm.round.argtypes = [C.c_double]


class Random:
    """The reference's Random (random.c), by handle."""

    def __init__(self, seed: int):
        self.h = lib().random_new(seed)

    def rand(self) -> int:
        return lib().random_rand(self.h)

    def next_double(self) -> float:
        return lib().random_nextDouble(self.h)

    def next_uint(self) -> int:
        return lib().random_nextUInt(self.h)

    @property
    def state(self) -> int:
        # struct _Random {guint seedState; guint initialSeed;} (random.c:15-18)
        return C.c_uint.from_address(self.h).value

    def free(self):
        if self.h:
            lib().random_free(self.h)
            self.h = None


def seed_chain(seed: int, n_hosts: int):
    """master.c:95 Random(seed) -> slave seed (master.c:417) -> slave Random
    (slave.c:182) -> scheduler seed (slave.c:198) -> node seeds (slave.c:301)."""
    master = Random(seed)
    slave_seed = master.next_uint()
    slave = Random(slave_seed)
    sched_seed = slave.next_uint()
    node = [slave.next_uint() for _ in range(n_hosts)]
    master.free()
    slave.free()
    return slave_seed, sched_seed, node


class _Ev(C.Structure):
    _fields_ = [("time", C.c_uint64), ("dst", C.c_uint32), ("src", C.c_uint32), ("seq", C.c_uint64),
                ("msg", C.c_uint64)]


_CMP = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p)


@_CMP
def _event_compare(a, b, _data):
    """event.c:110-153 (dst, then src, by host_compare = registration index)."""
    x, y = _Ev.from_address(a), _Ev.from_address(b)
    ka = (x.time, x.dst, x.src, x.seq)
    kb = (y.time, y.dst, y.src, y.seq)
    return (ka > kb) - (ka < kb)


def _digest_mix(pos, t, src, seq):
    from oracle import oracle as O  # the oracle's checksum term, so the two compare
    return O.digest_mix(pos, t, src, seq)


class RefPhold:
    """host_single rounds over the reference's PriorityQueue and Random.

    lat_ms / rel: V*V path latency (ms) and reliability of the direct paths;
    weights: PHOLD weights (None: uniform); vertex attachment by the reference
    rule over every vertex (topology.c:2327-2333)."""

    def __init__(self, n_hosts, lat_ms, rel, *, load=4, seed=1, end_time=500 * ONE_MS,
                 runahead_ms=0, weights=None, bootstrap_end=0):
        V = int(round(math.sqrt(len(lat_ms))))
        self.N, self.V, self.load = n_hosts, V, load
        self.lat = [float(x) for x in lat_ms]
        self.rel = [float(x) for x in rel]
        self.end_time, self.bootstrap_end = end_time, bootstrap_end
        self.runahead = runahead_ms * ONE_MS
        w = [1.0] * n_hosts if weights is None else [float(x) for x in weights]
        total = 0.0
        for x in w:  # test_phold.c:344
            total += x
        self.w, self.total = w, total
        _, _, node = seed_chain(seed, n_hosts)
        self.rng, self.vertex = [], []
        for i in range(n_hosts):
            r = Random(node[i])                     # host.c:176
            rd = r.next_double()                    # topology.c:2327
            self.vertex.append(int(_libm.round(float((V - 1) * rd))))
            self.rng.append(r)
        self.q = [lib().priorityqueue_new(C.cast(_event_compare, C.c_void_p), None, None)
                  for _ in range(n_hosts)]
        self.live = {}  # address -> _Ev: keeps the queued records alive
        self.evc = [0] * n_hosts
        self.pops = [0] * n_hosts
        self.digest = [0] * n_hosts
        self.stats = dict(rounds=0, pops=0, sends=0, null_dst=0, drop_reliability=0,
                          drop_endtime=0, bumped=0, same_round=0)
        self.S = self.E = 0
        self.jmin_ms = None
        self.next_min_jump = 0
        self.done = False

    # scheduler_push (scheduler.c:339-357) + host_single push (host_single.c:167-208)
    def _push(self, t, src, dst, seq, booting=False):
        if t >= self.end_time:
            self.stats["drop_endtime"] += 1
            return
        if src != dst and t < self.E:
            t = self.E
            self.stats["bumped"] += 1
        elif src == dst and t < self.E and not booting:
            self.stats["same_round"] += 1
        ev = _Ev(t, dst, src, seq, 0)
        a = C.addressof(ev)
        self.live[a] = ev
        lib().priorityqueue_push(self.q[dst], a)

    def _choose(self, h):
        r = self.rng[h].rand() / RAND_MAX  # random() routed to the host Random
        cumulative = 0.0
        for i in range(self.N):              # test_phold.c:166-170
            cumulative += self.w[i] / self.total
            if cumulative >= r:
                return i
        return None

    def _send(self, h, now):                 # worker.c:243-304
        d = self._choose(h)
        if d is None:
            self.stats["null_dst"] += 1
            return
        self.stats["sends"] += 1
        pair = self.vertex[h] * self.V + self.vertex[d]
        lat = self.lat[pair]
        ms = int(lat)                        # master.c:153 truncation of the discovered minimum
        self.jmin_ms = ms if self.jmin_ms is None else min(self.jmin_ms, ms)
        chance = self.rng[h].next_double()
        if not (now < self.bootstrap_end or chance <= self.rel[pair]):
            self.stats["drop_reliability"] += 1
            return
        seq = self.evc[h]
        self.evc[h] += 1
        self._push(now + math.ceil(lat * 1e6), h, d, seq)

    def boot(self):
        self.E = self.end_time               # pushed before the first round (scheduler.c:130)
        for h in range(self.N):
            seq = self.evc[h]
            self.evc[h] += 1
            self._push(0, h, h, seq, booting=True)
        self.S, self.E = 0, 1                # slave.c:431

    def _execute(self, ev):
        h = ev.dst
        pos = self.pops[h]
        self.pops[h] += 1
        self.stats["pops"] += 1
        self.digest[h] = (self.digest[h] + _digest_mix(pos, ev.time, ev.src, ev.seq)) & ((1 << 64) - 1)
        boot = ev.src == h and ev.seq == 0
        for _ in range(self.load if boot else 1):  # test_phold.c:234-239 / 310-312
            self._send(h, ev.time)

    def round(self):
        L = lib()
        for h in range(self.N):              # host_single.c:237-267
            while True:
                a = L.priorityqueue_peek(self.q[h])
                if not a or _Ev.from_address(a).time >= self.E:
                    break
                L.priorityqueue_pop(self.q[h])
                ev = self.live.pop(a)
                self._execute(ev)
        self.stats["rounds"] += 1
        m = SIMTIME_MAX                      # host_single.c:273-305
        for h in range(self.N):
            a = L.priorityqueue_peek(self.q[h])
            if a:
                m = min(m, _Ev.from_address(a).time)
        # master.c:450-480 with master_updateMinTimeJump (master.c:148-159)
        if self.jmin_ms is not None:
            self.next_min_jump = self.jmin_ms * ONE_MS
        jump = self.next_min_jump if self.next_min_jump > 0 else 10 * ONE_MS
        if self.runahead and jump < self.runahead:
            jump = self.runahead
        start = m
        end = min((m + jump) & ((1 << 64) - 1), self.end_time)  # SimulationTime wraps (master.c:470)
        self.S, self.E = start, end
        self.done = not start < end

    def run(self, max_rounds=1 << 62):
        while not self.done and self.stats["rounds"] < max_rounds:
            self.round()

    def host_state(self):
        return {"digest": np.array(self.digest, np.uint64), "pops": np.array(self.pops, np.uint64),
                "rng": np.array([r.state for r in self.rng], np.uint32),
                "ev": np.array(self.evc, np.uint64)}

    def close(self):
        L = lib()
        for q in self.q:
            L.priorityqueue_free(q)
        self.q = []
        for r in self.rng:
            r.free()
        self.live.clear()
