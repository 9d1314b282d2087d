"""CPU: where the reference's path cache makes discovery order-dependent, and
what sg_graph_paths reproduces.

The reference caches paths per source (topology.c:1338-1390) and, in an
undirected graph, answers a lookup (s, d) from the reverse entry d -> s when
s -> d is missing (topology.c:1986-1990).  A miss runs Dijkstra from s and
stores s -> t for every attached target t, except where t -> s is already
cached (_topology_shouldStorePath, topology.c:1306-1336); every store lowers
the global minimum path latency the window logic sees
(worker_updateMinTimeJump, topology.c:1374-1385).

Consequences, modelled below by a restatement of those rules (test code only):
  * path latencies depend on lookup order only through floating-point
    summation order: a reverse hit returns the d -> s sum, which can differ
    from the s -> d sum in the last bit (the ns delay is ceil(latency * 1e6),
    so this matters only at exact boundaries);
  * which sources run Dijkstra does: a lookup that hits a reverse entry runs
    nothing, so the discovered minimum can stay higher for the rest of the
    run.  Two orders of the same lookups (two workers racing in one round)
    can end with different minima, so the reference itself is order-dependent
    on undirected incomplete graphs;
  * complete graphs and prefer-direct adjacent pairs are not affected: each
    lookup stores (or finds) exactly its own pair's direct path;
  * directed graphs are affected more: the store guard and the post-run
    fallback ignore direction, so (s, t) can return the t -> s path.
sg_graph_paths gives every shortest-path lookup from s the minimum over all of
s's targets ("source-wide discovery"): the reference's value when s's lookup
runs its own Dijkstra, never above the reference's value under any order
(undirected graphs), and the true directed shortest path (directed graphs).
Every BASELINE config uses a complete graph, where the two agree exactly.
"""
import itertools

import pytest

import numpy as np

from shadow_amd import topology as T
from tests.test_topology import _graphml, _random_graph


class RefPathCache:
    """The reference's lookup / store rules for an all-attached graph whose
    shortest distances are `dist` (V x V) — test model, not product code."""

    def __init__(self, dist, adjacent, complete=False, prefer_direct=False, directed=False):
        self.dist, self.adj = dist, adjacent
        self.complete, self.prefer, self.directed = complete, prefer_direct, directed
        self.cache = {}
        self.min_lat = 0.0  # topology.c:1375: 0 = unset
        self.ran = set()

    def _store(self, s, t, lat, direct):  # topology.c:1306-1390
        if (s, t) in self.cache or (t, s) in self.cache:
            return
        if self.complete and not direct:
            return
        if self.prefer and not direct and self.adj[s][t]:
            return
        self.cache[(s, t)] = lat
        if self.min_lat == 0 or lat < self.min_lat:
            self.min_lat = lat

    def lookup(self, s, d):  # topology.c:1966-2047
        self.entry = (s, d)  # which cached entry answered (for the product check)
        p = self.cache.get((s, d))
        if p is None and not self.directed:
            self.entry = (d, s)
            p = self.cache.get((d, s))
        if p is not None:
            return p
        if self.complete or (self.prefer and self.adj[s][d]):
            self._store(s, d, self.dist[s][d], True)
        elif s == d:  # the path to self (topology.c:1545-1653), stored as non-direct
            self._store(s, s, self.dist[s][s], False)
        else:
            self.ran.add(s)
            for t in range(len(self.dist)):  # every attached target (topology.c:1676-1860)
                if t != s:
                    self._store(s, t, self.dist[s][t], False)
        p = self.cache.get((s, d))
        self.entry = (s, d) if p is not None else (d, s)
        return p if p is not None else self.cache.get((d, s))


def _line_graph():
    # v0 --10 ms-- v1 --1 ms-- v2
    return [(0, 1, 10.0, 0.0), (1, 2, 1.0, 0.0)]


def test_reverse_hit_makes_discovery_order_dependent():
    g = T.Graph(_graphml(3, _line_graph()))
    lat, _, disc, _ = g.paths()
    dist = lat.reshape(3, 3)
    adj = [[False] * 3 for _ in range(3)]
    finals = {}
    for order in ([(0, 1), (1, 0)], [(1, 0), (0, 1)]):
        ref = RefPathCache(dist, adj)
        got = [ref.lookup(s, d) for s, d in order]
        assert got == [10.0, 10.0]  # the latency itself: order-independent
        finals[tuple(order)] = (ref.min_lat, frozenset(ref.ran))
    # v0 first: only v0 runs, minimum 10 ms; v1 first: only v1 runs, minimum 1 ms
    assert finals[((0, 1), (1, 0))] == (10.0, frozenset({0}))
    assert finals[((1, 0), (0, 1))] == (1.0, frozenset({1}))
    # sg_graph_paths: each lookup knows its own source's minimum
    D = disc.reshape(3, 3)
    assert D[0, 1] == 10.0 and D[1, 0] == 1.0
    assert min(D[0, 1], D[1, 0]) == min(v[0] for v in finals.values())


def test_model_bounds_on_random_incomplete_graphs():
    """Over many lookup orders: latencies equal sg_graph_paths' in every order;
    the reference's running minimum is never below the running minimum of
    sg_graph_paths' discovered values, and equals it as long as every lookup's
    source has run its own Dijkstra (no lookup answered by a reverse entry
    for a source that never ran)."""
    rs = np.random.default_rng(7)
    n = 12
    g = T.Graph(_graphml(n, _random_graph(rs, n, 0.15)))
    lat, _, disc, _ = g.paths()
    dist, D = lat.reshape(n, n), disc.reshape(n, n)
    adj = [[False] * n for _ in range(n)]
    pairs = [(s, d) for s in range(n) for d in range(n) if s != d]
    differing = 0
    for trial in range(40):
        lookups = [pairs[i] for i in rs.choice(len(pairs), size=25, replace=False)]
        ref = RefPathCache(dist, adj)
        mine = np.inf
        exact = True
        for s, d in lookups:
            assert ref.lookup(s, d) in (dist[s, d], dist[d, s])
            if s not in ref.ran:
                exact = False  # answered by a reverse entry: s's Dijkstra never ran
            mine = min(mine, D[s, d])
            assert ref.min_lat >= mine
            if exact:
                assert ref.min_lat == mine
        differing += ref.min_lat != mine
    assert differing > 0  # the case the docs describe does occur
    # the two directions' sums agree to rounding
    assert np.allclose(dist, dist.T, rtol=1e-14, atol=0)


def test_complete_graphs_are_order_independent():
    """Complete graphs (every BASELINE config): every lookup stores or finds its
    own pair's direct path; the running minimum equals the running minimum of
    sg_graph_paths' discovered values in every order."""
    rs = np.random.default_rng(3)
    n = 6
    edges = [(a, b, float(rs.uniform(1, 50)), 0.0) for a in range(n) for b in range(a, n)]
    g = T.Graph(_graphml(n, edges))
    assert g.complete and not g.directed
    lat, _, disc, _ = g.paths()
    dist, D = lat.reshape(n, n), disc.reshape(n, n)
    adj = [[True] * n for _ in range(n)]
    pairs = [(s, d) for s in range(n) for d in range(n)]
    finals = set()
    for perm in itertools.islice(itertools.permutations(pairs[:7]), 0, 5040, 97):
        ref = RefPathCache(dist, adj, complete=True)
        mins = []
        for s, d in perm:
            assert ref.lookup(s, d) == dist[s, d]
            mins.append(ref.min_lat)
        assert np.array_equal(np.array(mins), np.minimum.accumulate([D[s, d] for s, d in perm]))
        finals.add(ref.min_lat)
    assert len(finals) == 1


def test_directed_graph_reverse_entry_is_returned():
    """Directed graphs: the store guard and the post-run fallback ignore the
    direction (topology.c:1312-1318, 2034-2036), so once t -> s is cached the
    lookup (s, t) runs Dijkstra from s, stores nothing for t and returns the
    t -> s path.  The reference's latency for (s, t) then depends on which
    direction was looked up first; sg_graph_paths returns the directed
    shortest path (the reference's value when s -> t comes first)."""
    edges = [(0, 1, 3.0, 0.0), (1, 2, 3.0, 0.0), (2, 0, 3.0, 0.0)]  # a one-way cycle
    g = T.Graph(_graphml(3, edges, directed=True))
    lat, _, _, _ = g.paths()
    dist = lat.reshape(3, 3)
    adj = [[False] * 3 for _ in range(3)]
    a = RefPathCache(dist, adj, directed=True)
    assert a.lookup(0, 1) == 3.0 and a.lookup(1, 0) == 3.0  # 1 -> 0 answered by 0 -> 1
    b = RefPathCache(dist, adj, directed=True)
    assert b.lookup(1, 0) == 6.0 and b.lookup(0, 1) == 6.0  # and the other way round
    assert (dist[0, 1], dist[1, 0]) == (3.0, 6.0)


def _cache_cases():
    rs = np.random.default_rng(11)
    n = 9
    und = _random_graph(rs, n, 0.2)
    yield "undirected", T.Graph(_graphml(n, und)), und, False, False
    yield "prefer-direct", T.Graph(_graphml(n, und, prefer="true")), und, True, False
    yield "directed", T.Graph(_graphml(n, _random_graph(rs, n, 0.25), directed=True)), None, False, True
    full = [(a, b, float(rs.uniform(1, 50)), 0.0) for a in range(5) for b in range(a, 5)]
    yield "complete", T.Graph(_graphml(5, full)), full, False, False


def test_product_path_cache_follows_the_model():
    """sg_path_cache (the CPU-worker driver's ordered discovery) against the
    model above on random lookup sequences, self lookups included: the same
    entry answers every lookup (forward or reverse) and the running minimum is
    the same after every lookup."""
    from shadow_amd import policy
    rs = np.random.default_rng(5)
    for name, g, edges, prefer, directed in _cache_cases():
        n = g.n_vertices
        lat, _, _, kind = g.paths()
        dist = lat.reshape(n, n)
        adj = [[False] * n for _ in range(n)]
        for a, b, _, _ in edges or []:
            adj[a][b] = True
            if not directed:
                adj[b][a] = True
        cfg = {"n_vertices": n, "paths": dict(latency_ms=lat, kind=kind, attached=np.ones(n, np.uint8),
                                               complete=g.complete, directed=g.directed)}
        for trial in range(20):
            pc = policy.PathCache(cfg)
            ref = RefPathCache(dist, adj, complete=g.complete, prefer_direct=prefer, directed=directed)
            for _ in range(30):
                s, d = (int(x) for x in rs.integers(0, n, 2))
                k, m = pc.lookup(s, d)
                want = ref.lookup(s, d)
                assert want is not None, (name, s, d)
                assert divmod(k, n) == ref.entry, (name, trial, s, d)
                assert lat[k] == want and m == ref.min_lat, (name, trial, s, d)
            pc.close()


# small incomplete graphs where the reference's lookup order changes the run
# (found by searching seeds: source-wide and ordered discovery differ)
ORDERED_CASES = [(2, 8), (7, 3), (11, 5), (33, 3)]


def ordered_case(seed, hosts, discovery):
    from shadow_amd import phold
    rs = np.random.default_rng(seed)
    n = int(rs.integers(4, 9))
    g = T.Graph(_graphml(n, _random_graph(rs, n, 0.2)))
    assert not g.complete
    return phold.topology_config(g, hosts, load=1, end_time_s=0.3, discovery=discovery, seed=seed + 1)


@pytest.mark.parametrize("seed,hosts", ORDERED_CASES)
def test_ordered_discovery_driver_matches_oracle(seed, hosts):
    """One CPU worker (shadow -w 1) under the host_single restatement: the
    driver's ordered discovery (sg_path_cache) and the oracle's restatement
    give the same run, and it is not the source-wide run."""
    from oracle import oracle as O
    from shadow_amd import policy
    runs = {}
    for disc in ("source", "ordered"):
        cfg = ordered_case(seed, hosts, disc)
        ref = O.Sim(cfg)
        ref.boot()
        ref.run()
        st, hs = ref.stats(), ref.host_state()
        r = policy.run_phold(cfg, 1, O.cpu_policy_ops(False, 1, hosts))
        assert (r["rounds"], r["bumped"], r["pops"]) == (st["rounds"], st["bumped"], st["pops"]), disc
        assert np.array_equal(r["digest"], hs["digest"]) and np.array_equal(r["ev"], hs["ev"]), disc
        runs[disc] = (st["rounds"], st["bumped"])
    assert runs["source"] != runs["ordered"]


def test_engine_refuses_ordered_discovery():
    from shadow_amd.engine import Engine
    with pytest.raises(ValueError, match="ordered path discovery"):
        Engine(ordered_case(7, 3, "ordered"))


def test_ordered_discovery_several_workers_runs():
    """With several workers the lookups reach the cache in whatever order the
    threads take (as in the reference): the run completes, every lookup is
    served under the driver's lock, and with one worker the run repeats
    exactly."""
    from oracle import oracle as O
    from shadow_amd import policy
    cfg = ordered_case(2, 8, "ordered")
    r4 = policy.run_phold(cfg, 4, O.cpu_policy_ops(False, 4, 8))
    assert r4["pops"] > 0 and r4["rounds"] > 0
    a = policy.run_phold(cfg, 1, O.cpu_policy_ops(False, 1, 8))
    b = policy.run_phold(cfg, 1, O.cpu_policy_ops(False, 1, 8))
    assert a["rounds"] == b["rounds"] and np.array_equal(a["digest"], b["digest"])


def test_ordered_discovery_stops_at_missing_path():
    """a send whose path the cache cannot return fails the run at
    the end of that round, instead of sending on a path the cache never
    returned and running on to endTime.  (sg_graph_paths refuses disconnected
    graphs, so the case is made by attaching no shortest-path target: every
    lookup that needs a Dijkstra run then stores nothing.)"""
    import ctypes as C
    from oracle import oracle as O
    from shadow_amd import _lib as L
    from shadow_amd import policy
    cfg = ordered_case(2, 8, "ordered")
    cfg["end_time"] = 100 * L.ONE_MS * 1000  # 100 s: a run that went on would take many rounds
    cfg["paths"] = dict(cfg["paths"], attached=np.zeros_like(np.asarray(cfg["paths"]["attached"])))
    lib = policy._bind()
    p, t, _keep = policy.phold_args(cfg)
    cache = policy.PathCache(cfg)
    ops = O.cpu_policy_ops(False, 2, cfg["n_hosts"])
    res = policy.SchedResult()
    rc = lib.sg_sched_run_phold_paths(C.byref(p), C.byref(t), cache.h, 2, policy.default_scheduler_seed(cfg),
                                      C.byref(ops), 1 << 40, C.byref(res), None, None, None, None)
    ops.free(ops.data)
    assert rc == L.SG_ERR_STATE
    assert "no path" in lib.sg_last_error().decode()
    assert res.rounds <= 2  # the boot round sends; the run ends after it
