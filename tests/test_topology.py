"""CPU: the GraphML → path-table stage (sg_topology.c) against the reference's
own data (the bundled topology and the C1 example's embedded topology, with
the survey's known-answer statistics) and against an independent shortest-path
implementation (scipy) on incomplete graphs."""
import json
import math
import os

import numpy as np
import pytest

from shadow_amd import _lib as L
from shadow_amd import phold
from shadow_amd import topology as T

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
KAT = json.load(open(os.path.join(GOLDEN, "kat.json")))


@pytest.fixture(scope="module")
def bundled():
    return T.Graph.from_file(T.BUNDLED)


def test_bundled_topology_matches_known_answers(bundled):
    k = KAT["bundled_topology"]
    g = bundled
    assert (g.n_vertices, g.n_edges) == (k["vertices"], k["edges"])
    assert g.complete and not g.directed and not g.prefers_direct
    src, dst, lat, loss = g.edges()
    assert lat.min() == k["latency_min_ms"] and lat.max() == k["latency_max_ms"]
    assert np.median(lat) == k["latency_median_ms"]
    assert set(loss.tolist()) == {k["edge_packetloss"]}
    assert all(g.vertex(i)["packetloss"] == k["vertex_packetloss"] for i in range(g.n_vertices))
    assert int((src == dst).sum()) == g.n_vertices  # complete with self-loops
    # ceil(latency * 1e6) rounds up on exactly 248 edges
    up = sum(math.ceil(x * 1e6) != round(x * 1e6) for x in lat.tolist())
    assert up == k["ceil_roundup_edges"]


def test_bundled_paths_are_direct_and_symmetric(bundled):
    g = bundled
    lat, rel, disc, kind = g.paths()
    V = g.n_vertices
    assert (kind == T.PATH_DIRECT).all()
    assert np.array_equal(lat.reshape(V, V), lat.reshape(V, V).T)
    # direct path: 1 * (1 - 0.0) * (1 - 0.0) * (1 - 0.005) (topology.c:1887-1921)
    assert set(rel.tolist()) == {1.0 * (1.0 - 0.0) * (1.0 - 0.0) * (1.0 - 0.005)}
    assert np.array_equal(disc, lat)
    src, dst, elat, _ = g.edges()
    m = lat.reshape(V, V)
    assert all(m[a, b] == x and m[b, a] == x for a, b, x in zip(src.tolist(), dst.tolist(), elat.tolist()))
    # the device tables agree with sg_build_paths' direct-path restatement
    d1, k1, j1 = T.path_tables(lat, rel, disc)
    d2, k2, j2 = phold.build_paths(lat, np.full(V * V, 0.005), np.zeros(V))
    assert np.array_equal(d1, d2) and np.array_equal(k1, k2) and np.array_equal(j1, j2)


def test_known_delay_values():
    for ms, ns in KAT["ceil_delay_ns"]:
        d, _, _ = T.path_tables(np.array([ms]), np.array([1.0]))
        assert int(d[0]) == ns
    for ms, jm in KAT["trunc_ms"]:
        _, _, j = T.path_tables(np.array([ms]), np.array([1.0]))
        assert int(j[0]) == jm


def test_c1_embedded_topology():
    g = T.Graph.from_file(T.C1_EMBEDDED)
    assert (g.n_vertices, g.n_edges, g.complete) == (1, 1, True)
    lat, rel, disc, kind = g.paths()
    assert lat[0] == 50.0 and rel[0] == 1.0 * (1.0 - 0.0) * (1.0 - 0.0) * (1.0 - 0.01)
    d, k, j = T.path_tables(lat, rel, disc)
    assert int(d[0]) == 50_000_000 and int(j[0]) == 50
    assert int(k[0]) == L.lib().sg_keep_threshold(rel[0])


def _graphml(n, edges, directed=False, vloss=None, prefer=None, extra_node=None):
    out = ['<?xml version="1.0"?><graphml>',
           '<key attr.name="latency" attr.type="double" for="edge" id="l"/>',
           '<key attr.name="packetloss" attr.type="double" for="edge" id="p"/>',
           '<key attr.name="packetloss" attr.type="double" for="node" id="vp"/>',
           '<key attr.name="type" attr.type="string" for="node" id="t"/>',
           '<key attr.name="countrycode" attr.type="string" for="node" id="c"/>',
           '<key attr.name="ip" attr.type="string" for="node" id="ip"/>',
           '<key attr.name="preferdirectpaths" attr.type="string" for="graph" id="g"/>',
           f'<graph edgedefault="{"directed" if directed else "undirected"}">']
    if prefer is not None:
        out.append(f'<data key="g">{prefer}</data>')
    for i in range(n):
        body = ""
        if vloss is not None:
            body += f'<data key="vp">{float(vloss[i])!r}</data>'
        if extra_node:
            for k, v in (extra_node(i) or {}).items():
                body += f'<data key="{k}">{v}</data>'
        out.append(f'<node id="v{i}">{body}</node>')
    for a, b, lat, loss in edges:
        out.append(f'<edge source="v{a}" target="v{b}"><data key="l">{lat!r}</data>'
                   f'<data key="p">{loss!r}</data></edge>')
    out.append("</graph></graphml>")
    return "\n".join(out)


def _random_graph(rs, n, p):
    edges = []
    for a in range(n):  # a ring keeps it connected
        edges.append((a, (a + 1) % n, float(rs.uniform(1, 50)), float(rs.uniform(0, 0.05))))
    for a in range(n):
        for b in range(a + 2, n):
            if (a, b) != (0, n - 1) and rs.random() < p:  # no parallel edges
                edges.append((a, b, float(rs.uniform(1, 50)), float(rs.uniform(0, 0.05))))
    return edges


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_shortest_paths_against_scipy(seed):
    from scipy.sparse import csr_matrix
    from scipy.sparse.csgraph import dijkstra
    rs = np.random.default_rng(seed)
    n = 40
    edges = _random_graph(rs, n, 0.08)
    vloss = rs.uniform(0, 0.02, n)
    g = T.Graph(_graphml(n, edges, vloss=vloss))
    assert not g.complete
    lat, rel, disc, kind = g.paths()
    W = np.full((n, n), np.inf)
    for a, b, l, _ in edges:
        W[a, b] = W[b, a] = min(W[a, b], l)
    ref = dijkstra(csr_matrix(np.where(np.isinf(W), 0, W)), directed=False)
    m = lat.reshape(n, n)
    off = ~np.eye(n, dtype=bool)
    assert np.allclose(m[off], ref[off], rtol=1e-12)
    assert (kind.reshape(n, n)[off] == T.PATH_SHORTEST).all()
    assert (kind.reshape(n, n)[~off] == T.PATH_SELF).all()
    # path reliability: rebuild each path from scipy's predecessors (unique with random weights)
    _, pred = dijkstra(csr_matrix(np.where(np.isinf(W), 0, W)), directed=False, return_predecessors=True)
    loss = {}
    for a, b, l, p in edges:
        loss[(a, b)] = loss[(b, a)] = p
    R = rel.reshape(n, n)
    for s in range(0, n, 7):
        for t in range(n):
            if s == t:
                continue
            path = [t]
            while path[-1] != s:
                path.append(pred[s, path[-1]])
            path = path[::-1]
            r = 1.0 * (1.0 - vloss[s]) * (1.0 - vloss[t])
            for u, v in zip(path, path[1:]):
                r *= (1.0 - loss[(u, v)])
            assert R[s, t] == r, (s, t)
    # source-wide discovery: every shortest-path lookup from s knows the min over s's targets
    D = disc.reshape(n, n)
    for s in range(n):
        assert np.all(D[s, off[s]] == m[s, off[s]].min())


def test_self_path_rule():
    # v0 -- v1 (10 ms, loss .1), v0 -- v2 (4 ms, loss .2), v1 -- v2 (7 ms)
    edges = [(0, 1, 10.0, 0.1), (0, 2, 4.0, 0.2), (1, 2, 7.0, 0.0)]
    g = T.Graph(_graphml(3, edges, vloss=[0.5, 0.5, 0.5]))
    lat, rel, disc, kind = g.paths()
    # topology.c:1545-1653: min incident edge twice, no vertex loss
    assert kind[0] == T.PATH_SELF and lat[0] == 2.0 * 4.0 and rel[0] == (1.0 - 0.2) * (1.0 - 0.2)
    assert lat[1 * 3 + 1] == 2.0 * 7.0
    # v1 -> v0 goes through v2 (7 + 4 = 11 > 10? no: direct 10 is shorter)
    assert lat[1 * 3 + 0] == 10.0 and kind[1 * 3 + 0] == T.PATH_SHORTEST
    assert rel[1 * 3 + 0] == 1.0 * (1.0 - 0.5) * (1.0 - 0.5) * (1.0 - 0.1)


def test_prefer_direct_paths():
    # v0 -- v1 is 100 ms directly but 2 ms through v2
    edges = [(0, 1, 100.0, 0.0), (0, 2, 1.0, 0.0), (2, 1, 1.0, 0.0)]
    lat0, _, disc0, kind0 = T.Graph(_graphml(3, edges)).paths()
    assert lat0[1] == 2.0 and kind0[1] == T.PATH_SHORTEST
    lat1, _, disc1, kind1 = T.Graph(_graphml(3, edges, prefer="true")).paths()
    assert lat1[1] == 100.0 and kind1[1] == T.PATH_DIRECT
    for val in ("yes", "1", "TRUE"):
        assert T.Graph(_graphml(3, edges, prefer=val)).prefers_direct
    assert not T.Graph(_graphml(3, edges, prefer="false")).prefers_direct


def test_zero_latency_path_becomes_one_ms():
    edges = [(0, 1, 0.0, 0.0), (1, 2, 5.0, 0.0)]
    lat, _, _, kind = T.Graph(_graphml(3, edges)).paths()
    assert lat[0 * 3 + 1] == 1.0 and kind[1] == T.PATH_SHORTEST  # topology.c:1848-1852


def test_directed_graph():
    edges = [(0, 1, 3.0, 0.0), (1, 2, 3.0, 0.0), (2, 0, 3.0, 0.0)]
    g = T.Graph(_graphml(3, edges, directed=True))
    lat, _, _, _ = g.paths()
    m = lat.reshape(3, 3)
    assert m[0, 1] == 3.0 and m[1, 0] == 6.0  # only forward along the cycle


def test_completeness_counts_self_loops_once():
    n = 3
    full = [(a, b, 1.0, 0.0) for a in range(n) for b in range(a, n)]
    assert T.Graph(_graphml(n, full)).complete
    assert not T.Graph(_graphml(n, [e for e in full if e[0] != e[1] or e[0] != 2])).complete


def test_attach_without_hints_matches_random_rule():
    g = T.Graph(_graphml(7, [(a, (a + 1) % 7, 1.0, 0.0) for a in range(7)]))
    _, _, node = phold.seed_chain(1, 500)
    v1, r1 = g.attach(node)
    v2, r2 = phold.attach(node, 7, L.SG_ATTACH_RANDOM)
    assert np.array_equal(v1, v2) and np.array_equal(r1, r2)


def test_attach_hints():
    nodes = {0: {"c": "US", "t": "relay", "ip": "10.0.0.1"}, 1: {"c": "US", "t": "client", "ip": "10.0.1.1"},
             2: {"c": "DE", "t": "relay", "ip": "11.0.0.1"}, 3: {"c": "DE", "ip": "0.0.0.0"},
             4: {"c": "FR", "ip": "10.0.0.200"}}
    g = T.Graph(_graphml(5, [(a, (a + 1) % 5, 1.0, 0.0) for a in range(5)], extra_node=lambda i: nodes[i]))
    seeds = np.array([12345] * 6, np.uint32)
    hints = [{"countrycode": "DE", "type": "relay"},   # country+type: only v2, one draw
             {"countrycode": "de"},                    # case-insensitive, v2 or v3
             {"ip": "10.0.1.1"},                       # exact IP match: v1, one draw
             {"ip": "10.0.0.7"},                       # longest prefix over all: v0, no draw
             {"countrycode": "ZZ"},                    # no match: all vertices, one draw
             {"type": "client", "ip": "12.0.0.1"}]     # type set; LPM inside it: v1, no draw
    v, r = g.attach(seeds, hints)
    # an exact IP match wins over every filter (topology.c:2133-2159)
    v2, r2 = g.attach(seeds[:1], [{"type": "client", "ip": "11.0.0.1"}])
    assert v2[0] == 2 and r2[0] != seeds[0]
    assert v[0] == 2 and v[2] == 1 and v[3] == 0 and v[5] == 1
    assert v[1] in (2, 3)
    drew = r != seeds
    assert drew.tolist() == [True, True, True, False, True, False]
    # the draw picks round((n-1) * nextDouble) among the candidates in vertex order
    st = np.uint32(12345)
    x = np.array([st], np.uint32)
    dbl = L.lib().sg_random_next_double(x.ctypes.data_as(L.C.POINTER(L.C.c_uint32)))
    assert v[1] == [2, 3][int(round(1 * dbl))]
    assert v[4] == int(round(4 * dbl))


def test_c3_shape_config_builds():
    cfg = phold.c3_config(n_relays=200, n_clients=800, end_time_s=0.2)
    assert cfg["n_hosts"] == 1000 and cfg["n_vertices"] == 183
    assert cfg["host_vertex"].max() < 183
    assert (cfg["keep_max"] == L.lib().sg_keep_threshold(0.995)).all()


def test_malformed_graphml_rejected():
    for bad in ["", "<graphml></graphml>", "<graphml><graph><node/></graph></graphml>",
                _graphml(2, [(0, 1, 1.0, 0.0)]).replace('target="v1"', 'target="nope"')]:
        with pytest.raises(L.SgError):
            T.Graph(bad)
