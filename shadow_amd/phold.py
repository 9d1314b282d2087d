"""Synthetic PHOLD workloads (BASELINE.json configs) built with libshadowgpu's
host-side restatements of the reference arithmetic.

A config is a plain dict: scalar parameters + the tables the device engine
consumes (host vertex, per-host rand_r state after attachment, V*V delay /
keep-threshold / truncated-latency matrices, PHOLD weight thresholds).

PHOLD model, one committed event at host h, time t:
  boot event (self, t=0, id 0) sends `load` messages; a message event sends one:
    x = rand_r(h) -> destination (test_phold.c:160-178, or the probe's floor rule)
    c = rand_r(h) -> kept iff bootstrapping or c/RAND_MAX <= reliability (worker.c:268-273)
    deliver = t + ceil(latency_ms * 1e6), id = h.eventCounter++   (worker.c:275-297)
    scheduler_push: dropped at >= endTime, bumped to the barrier if inter-host
"""
from __future__ import annotations

import ctypes as C
import math

import numpy as np

from . import _lib as L


# ------------------------------------------------------------- primitives ----
def rand_r_stream(seed: int, n: int) -> np.ndarray:
    st = C.c_uint32(seed)
    f = L.lib().sg_rand_r
    return np.array([f(C.byref(st)) for _ in range(n)], dtype=np.int64)


def seed_chain(seed: int, n_hosts: int):
    node = np.zeros(max(n_hosts, 1), np.uint32)
    a, b = C.c_uint32(), C.c_uint32()
    L.check(L.lib().sg_seed_chain(seed, n_hosts, C.byref(a), C.byref(b), node))
    return a.value, b.value, node[:n_hosts]


def attach(node_seeds, n_vertices: int, rule: int):
    n = len(node_seeds)
    v = np.zeros(max(n, 1), np.uint32)
    r = np.zeros(max(n, 1), np.uint32)
    L.check(L.lib().sg_attach_hosts(n, n_vertices, rule,
                                    np.ascontiguousarray(node_seeds, np.uint32), v, r))
    return v[:n], r[:n]


def keep_threshold(rel: float) -> int:
    return L.lib().sg_keep_threshold(rel)


def build_paths(latency_ms, edge_loss, vertex_loss=None):
    lat = np.ascontiguousarray(latency_ms, np.float64).ravel()
    V = int(round(math.sqrt(lat.size)))
    assert V * V == lat.size, "latency matrix must be V*V"
    el = np.ascontiguousarray(edge_loss, np.float64).ravel()
    d = np.zeros(V * V, np.uint64)
    k = np.zeros(V * V, np.int32)
    j = np.zeros(V * V, np.uint32)
    vl = None if vertex_loss is None else np.ascontiguousarray(vertex_loss, np.float64)
    L.check(L.lib().sg_build_paths(V, lat, el, None if vl is None else vl.ctypes.data, d, k, j))
    return d, k, j


def weight_thresholds(weights) -> np.ndarray:
    w = np.ascontiguousarray(weights, np.float64)
    out = np.zeros(len(w), np.int32)
    L.check(L.lib().sg_build_weight_thresholds(len(w), w, out))
    return out


def lognormal_topology(V: int, seed: int, median_ms: float, sigma: float, min_ms: float,
                       edge_loss: float = 0.0):
    lat = np.zeros(V * V, np.float64)
    el = np.zeros(V * V, np.float64)
    L.check(L.lib().sg_topology_lognormal(V, seed, median_ms, sigma, min_ms, edge_loss, lat, el))
    return lat, el


# --------------------------------------------------------------- configs -----
def make_config(*, n_hosts, latency_ms, edge_loss, vertex_loss=None, load=16, seed=1,
                end_time_s=10.0, dst_rule=L.SG_DST_WEIGHTS, attach_rule=L.SG_ATTACH_RANDOM,
                window_rule=L.SG_WINDOW_DISCOVERED, fixed_jump_ms=0, runahead_ms=0,
                bootstrap_end=0, weights=None, keep_override=None, delay_override=None,
                name="phold"):
    lat = np.ascontiguousarray(latency_ms, np.float64).ravel()
    V = int(round(math.sqrt(lat.size)))
    _, _, node = seed_chain(seed, n_hosts)
    vertex, rng = attach(node, V, attach_rule)
    delay, keep, jump = build_paths(lat, edge_loss, vertex_loss)
    if keep_override is not None:
        keep = np.ascontiguousarray(keep_override, np.int32)
    if delay_override is not None:
        delay = np.ascontiguousarray(delay_override, np.uint64)
    wt = None
    if dst_rule == L.SG_DST_WEIGHTS:
        wt = weight_thresholds(np.ones(n_hosts) if weights is None else weights)
    return dict(
        name=name, n_hosts=n_hosts, n_vertices=V, load=load, seed=seed,
        dst_rule=dst_rule, window_rule=window_rule, attach_rule=attach_rule,
        end_time=int(round(end_time_s * 1e9)), bootstrap_end=int(bootstrap_end),
        fixed_jump=int(fixed_jump_ms * L.ONE_MS), runahead_min=int(runahead_ms * L.ONE_MS),
        host_vertex=vertex, host_rng=rng, delay_ns=delay, keep_max=keep, jump_ms=jump,
        weight_thresh=wt)


def probe_config(n_hosts=1000, jump_ms=5, V=8, load=16, rel=0.99, end_time_s=2.0):
    """The survey's probe workload (SURVEY.md §0 finding 2): uniform-floor
    destinations, vertex = index mod 8, latency 5 + 3.37*((7i+3j) mod 8) ms,
    reliability 0.99, fixed window.  Its reference trace hashes are pinned in
    tests/golden/probe_hashes.json."""
    lat = np.zeros(V * V)
    for i in range(V):
        for j in range(V):
            lat[i * V + j] = 5.0 + 3.37 * ((i * 7 + j * 3) % V)
    delay = np.array([math.ceil(x * 1_000_000) for x in lat], np.uint64)
    keep = np.full(V * V, keep_threshold(rel), np.int32)
    return make_config(n_hosts=n_hosts, latency_ms=lat, edge_loss=np.zeros(V * V), load=load,
                       seed=1, end_time_s=end_time_s, dst_rule=L.SG_DST_UNIFORM_FLOOR,
                       attach_rule=L.SG_ATTACH_MODULO, window_rule=L.SG_WINDOW_FIXED,
                       fixed_jump_ms=jump_ms, keep_override=keep, delay_override=delay,
                       name=f"probe-{n_hosts}-j{jump_ms}")


def c2_config(n_hosts=10_000, end_time_s=10.0, load=16):
    """BASELINE configs[1]: PHOLD 10k hosts x 16, uniform 50 ms full mesh (one
    vertex, as phold.test.shadow.config.xml), loss 0."""
    return make_config(n_hosts=n_hosts, latency_ms=np.array([50.0]), edge_loss=np.zeros(1),
                       load=load, end_time_s=end_time_s, name=f"phold-c2-{n_hosts}")


def c4_config(n_hosts=1_000_000, V=1024, end_time_s=10.0, load=16, seed_topology=4):
    """BASELINE configs[3]: PHOLD 1M hosts x 16, skewed (log-normal) latency over
    V vertices, minimum 1 ms, runahead -r 1."""
    lat, el = lognormal_topology(V, seed_topology, median_ms=30.0, sigma=0.9, min_ms=1.0)
    return make_config(n_hosts=n_hosts, latency_ms=lat, edge_loss=el, load=load,
                       end_time_s=end_time_s, runahead_ms=1, name=f"phold-c4-{n_hosts}")


def _lossy_mesh(V, seed_topology, loss):
    lat, _ = lognormal_topology(V, seed_topology, median_ms=40.0, sigma=0.7, min_ms=2.0)
    rs = np.random.default_rng(seed_topology)  # input generation only
    el = rs.uniform(loss[0], loss[1], size=(V, V))
    el = np.triu(el) + np.triu(el, 1).T
    return lat, el.ravel()


def lossy_config(n_hosts=100_000, V=256, end_time_s=10.0, load=8, loss=(0.005, 0.05),
                 seed_topology=5):
    """PHOLD on configs[4]'s lossy links (edge loss uniform in [0.005, 0.05]);
    every send draws the host's reliability chance."""
    lat, el = _lossy_mesh(V, seed_topology, loss)
    return make_config(n_hosts=n_hosts, latency_ms=lat, edge_loss=el, load=load,
                       end_time_s=end_time_s, name=f"lossy-phold-{n_hosts}")


def c5_config(n_hosts=100_000, V=256, fanout=8, msgs=64, start_ms=1.0, interval_ms=5.0,
              end_time_s=10.0, loss=(0.005, 0.05), seed_topology=5, seed=1):
    """BASELINE configs[4]: Bitcoin-style gossip over lossy links.  Message m of
    `msgs` originates at host floor(m*N/msgs) at start + m*interval; a host's
    first receipt of a message forwards it to `fanout` drawn peers (each send
    through worker_sendPacket: reliability draw, then the drop test,
    worker.c:267-279); later receipts are dropped by the host's seen set.
    Links: log-normal latency (median 40 ms, min 2 ms) over V vertices, edge
    loss uniform in [0.005, 0.05]."""
    lat, el = _lossy_mesh(V, seed_topology, loss)
    cfg = make_config(n_hosts=n_hosts, latency_ms=lat, edge_loss=el, load=fanout, seed=seed,
                      end_time_s=end_time_s, name=f"gossip-c5-{n_hosts}")
    cfg.update(workload=L.SG_WORKLOAD_GOSSIP, gossip_msgs=msgs,
               gossip_start=int(round(start_ms * L.ONE_MS)),
               gossip_interval=int(round(interval_ms * L.ONE_MS)))
    return cfg


def topology_config(graph, n_hosts, *, load=16, seed=1, end_time_s=10.0, hints=None,
                    dst_rule=L.SG_DST_WEIGHTS, window_rule=L.SG_WINDOW_DISCOVERED, runahead_ms=0,
                    fixed_jump_ms=0, bootstrap_end=0, weights=None, name=None, discovery="source"):
    """PHOLD on a GraphML topology (shadow_amd.topology.Graph): hosts attached
    by topology_attach from their node seeds (host.c:176, topology.c:2094-2369),
    paths resolved as topology.c would (direct, shortest or self), the jump table
    carrying each lookup's discovered minimum latency (topology.c:1374-1385).
    discovery="ordered" also carries what the reference's lazy path cache needs
    (cfg["paths"]): the CPU-worker driver (policy.run_phold) and the oracle then
    replay the cache in their lookup order, which is the reference's with one
    worker; the device engine keeps the source-wide jump table and refuses it."""
    from . import topology as T
    if discovery not in ("source", "ordered"):
        raise ValueError(f"discovery must be 'source' or 'ordered', not {discovery!r}")
    _, _, node = seed_chain(seed, n_hosts)
    vertex, rng = graph.attach(node, hints)
    attached = np.zeros(graph.n_vertices, bool)
    attached[vertex] = True
    lat, rel, disc, kind = graph.paths(attached)
    delay, keep, jump = T.path_tables(lat, rel, disc)
    wt = None
    if dst_rule == L.SG_DST_WEIGHTS:
        wt = weight_thresholds(np.ones(n_hosts) if weights is None else weights)
    return dict(
        name=name or f"phold-topology-{n_hosts}", n_hosts=n_hosts, n_vertices=graph.n_vertices,
        load=load, seed=seed, dst_rule=dst_rule, window_rule=window_rule,
        attach_rule=L.SG_ATTACH_RANDOM, end_time=int(round(end_time_s * 1e9)),
        bootstrap_end=int(bootstrap_end), fixed_jump=int(fixed_jump_ms * L.ONE_MS),
        runahead_min=int(runahead_ms * L.ONE_MS), host_vertex=vertex, host_rng=rng,
        delay_ns=delay, keep_max=keep, jump_ms=jump, weight_thresh=wt,
        discovery=discovery,
        paths=dict(latency_ms=lat, kind=kind, attached=attached.astype(np.uint8), complete=graph.complete,
                   directed=graph.directed) if discovery == "ordered" else None)


def c1_config(end_time_s=3600.0, load=16, seed=1):
    """BASELINE configs[0] shape without tgen (the plugin is not available
    offline): the example config's two hosts ("server", "client") on its
    embedded one-vertex topology (50 ms self-loop, loss 0.01), stoptime 3600 s,
    PHOLD traffic between them."""
    from . import topology as T
    g = T.Graph.from_file(T.C1_EMBEDDED)
    return topology_config(g, 2, load=load, seed=seed, end_time_s=end_time_s,
                           name="c1-example-2")


def c3_config(n_relays=2000, n_clients=8000, end_time_s=10.0, load=4, seed=1):
    """BASELINE configs[2] shape without tgen (the plugin is not available
    offline): 2k relay + 8k client hosts on the bundled topology, PHOLD traffic
    over the resulting paths.  Every bundled vertex is typed "cluster", so the
    relays carry country-code hints instead (round-robin over the topology's
    own codes; topology.c:2180-2192 filters on them) and the clients none."""
    from . import topology as T
    g = T.Graph.from_file(T.BUNDLED)
    codes = sorted({g.vertex(i)["countrycode"] for i in range(g.n_vertices)} - {None})
    n = n_relays + n_clients
    hints = [{"countrycode": codes[i % len(codes)]} if i < n_relays else None for i in range(n)]
    return topology_config(g, n, load=load, seed=seed, end_time_s=end_time_s, hints=hints,
                           name=f"tor-shape-c3-{n}")


def tiny_config(n_hosts=64, V=4, load=4, end_time_s=0.5, loss=0.02, runahead_ms=0,
                window_rule=L.SG_WINDOW_DISCOVERED, dst_rule=L.SG_DST_WEIGHTS, seed=7,
                weights=None, min_ms=1.0):
    lat, el = lognormal_topology(V, seed + 100, median_ms=10.0, sigma=0.8, min_ms=min_ms,
                                 edge_loss=loss)
    return make_config(n_hosts=n_hosts, latency_ms=lat, edge_loss=el, load=load, seed=seed,
                       end_time_s=end_time_s, runahead_ms=runahead_ms, window_rule=window_rule,
                       dst_rule=dst_rule, weights=weights, name=f"tiny-{n_hosts}")
