"""GraphML topologies → device path tables (include/shadowgpu.h §1b,
shadow_amd/csrc/sg_topology.c).

Mirrors the routing/topology.c surface the scheduler's hot path depends on:
load a GraphML topology (topology.c:554-800), attach hosts to vertices
(topology_attach, topology.c:2094-2369), and resolve every vertex pair's path
latency/reliability (topology_getLatency / topology_getReliability,
topology.c:1969-2087).  The resulting V*V tables feed the device engine's
one-lookup-per-send path records.
"""
from __future__ import annotations

import ctypes as C
import lzma
import os

import numpy as np

from . import _lib as L

PATH_DIRECT, PATH_SHORTEST, PATH_SELF = 0, 1, 2


class GraphDesc(C.Structure):
    _fields_ = [("n_vertices", C.c_uint32), ("n_edges", C.c_uint32), ("directed", C.c_int32),
                ("complete", C.c_int32), ("prefers_direct", C.c_int32),
                ("min_edge_latency_ms", C.c_double), ("max_edge_latency_ms", C.c_double)]


class VertexDesc(C.Structure):
    _fields_ = [(n, C.c_char_p) for n in ("id", "ip", "citycode", "countrycode", "geocode", "type")] + \
               [("packetloss", C.c_double), ("has_packetloss", C.c_int32),
                ("bandwidth_down", C.c_uint64), ("bandwidth_up", C.c_uint64)]


class AttachHint(C.Structure):
    _fields_ = [(n, C.c_char_p) for n in ("ip", "citycode", "countrycode", "geocode", "type")]


def _bind():
    lib = L.lib()
    if getattr(lib, "_topo_bound", False):
        return lib
    vp = C.c_void_p
    lib.sg_graphml_load.argtypes = [C.c_char_p, C.c_uint64, C.POINTER(vp)]
    lib.sg_graph_free.argtypes = [vp]
    lib.sg_graph_info.argtypes = [vp, C.POINTER(GraphDesc)]
    lib.sg_graph_vertex.argtypes = [vp, C.c_uint32, C.POINTER(VertexDesc)]
    lib.sg_graph_edge.argtypes = [vp, C.c_uint32, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
                                  C.POINTER(C.c_double), C.POINTER(C.c_double)]
    lib.sg_graph_attach.argtypes = [vp, C.c_uint32, vp, L.u32p, L.u32p]
    lib.sg_graph_paths.argtypes = [vp, vp, L.f64p, L.f64p, vp, vp]
    lib.sg_build_path_tables.argtypes = [C.c_uint32, L.f64p, L.f64p, vp, L.u64p, L.i32p, L.u32p]
    lib._topo_bound = True
    return lib


def read_text(path: str) -> str:
    """A GraphML file, xz-compressed or plain."""
    if path.endswith(".xz"):
        with lzma.open(path) as f:
            return f.read().decode()
    with open(path) as f:
        return f.read()


class Graph:
    """A parsed GraphML topology (sg_graph)."""

    def __init__(self, text: str):
        lib = _bind()
        raw = text.encode()
        h = C.c_void_p()
        L.check(lib.sg_graphml_load(raw, len(raw), C.byref(h)))
        self.h = h
        d = GraphDesc()
        L.check(lib.sg_graph_info(h, C.byref(d)))
        self.n_vertices = d.n_vertices
        self.n_edges = d.n_edges
        self.directed = bool(d.directed)
        self.complete = bool(d.complete)
        self.prefers_direct = bool(d.prefers_direct)
        self.min_edge_latency_ms = d.min_edge_latency_ms
        self.max_edge_latency_ms = d.max_edge_latency_ms

    @classmethod
    def from_file(cls, path: str) -> "Graph":
        return cls(read_text(path))

    def close(self):
        if getattr(self, "h", None):
            L.lib().sg_graph_free(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def vertex(self, i: int) -> dict:
        v = VertexDesc()
        L.check(_bind().sg_graph_vertex(self.h, i, C.byref(v)))
        s = lambda b: None if b is None else b.decode()  # noqa: E731
        return {"id": s(v.id), "ip": s(v.ip), "citycode": s(v.citycode), "countrycode": s(v.countrycode),
                "geocode": s(v.geocode), "type": s(v.type),
                "packetloss": v.packetloss if v.has_packetloss else None,
                "bandwidth_down": int(v.bandwidth_down), "bandwidth_up": int(v.bandwidth_up)}

    def edges(self):
        """(src, dst, latency_ms, packetloss) arrays in edge order."""
        n = self.n_edges
        src = np.zeros(n, np.uint32)
        dst = np.zeros(n, np.uint32)
        lat = np.zeros(n)
        loss = np.zeros(n)
        a, b, l, p = C.c_uint32(), C.c_uint32(), C.c_double(), C.c_double()
        f = _bind().sg_graph_edge
        for i in range(n):
            L.check(f(self.h, i, C.byref(a), C.byref(b), C.byref(l), C.byref(p)))
            src[i], dst[i], lat[i], loss[i] = a.value, b.value, l.value, p.value
        return src, dst, lat, loss

    def attach(self, rng_states, hints=None):
        """topology_attach for every host in registration order.  rng_states are
        the hosts' Random states (advanced in place by the draw); hints a list of
        dicts with keys ip/citycode/countrycode/geocode/type, or None."""
        rng = np.ascontiguousarray(rng_states, np.uint32).copy()
        n = len(rng)
        out = np.zeros(max(n, 1), np.uint32)
        harr = None
        keep = []
        if hints is not None:
            harr = (AttachHint * n)()
            for i, h in enumerate(hints):
                for k in ("ip", "citycode", "countrycode", "geocode", "type"):
                    v = (h or {}).get(k)
                    if v is not None:
                        b = v.encode()
                        keep.append(b)
                        setattr(harr[i], k, b)
        L.check(_bind().sg_graph_attach(self.h, n, None if harr is None else C.cast(harr, C.c_void_p),
                                        rng if n else np.zeros(1, np.uint32), out))
        return out[:n], rng

    def paths(self, attached=None):
        """Every vertex pair's path: latency_ms, reliability, discovered_ms, kind (V*V)."""
        V = self.n_vertices
        lat = np.zeros(V * V)
        rel = np.zeros(V * V)
        disc = np.zeros(V * V)
        kind = np.zeros(V * V, np.uint8)
        att = None
        if attached is not None:
            att = np.ascontiguousarray(np.asarray(attached, bool).astype(np.uint8))
            assert att.size == V
        L.check(_bind().sg_graph_paths(self.h, None if att is None else att.ctypes.data, lat, rel,
                                       disc.ctypes.data, kind.ctypes.data))
        return lat, rel, disc, kind


def path_tables(latency_ms, reliability, discovered_ms=None):
    """Device tables: delay_ns (ceil), keep_max, jump_ms (sg_build_path_tables)."""
    lat = np.ascontiguousarray(latency_ms, np.float64).ravel()
    rel = np.ascontiguousarray(reliability, np.float64).ravel()
    V = int(round(np.sqrt(lat.size)))
    d = np.zeros(V * V, np.uint64)
    k = np.zeros(V * V, np.int32)
    j = np.zeros(V * V, np.uint32)
    disc = None if discovered_ms is None else np.ascontiguousarray(discovered_ms, np.float64).ravel()
    L.check(_bind().sg_build_path_tables(V, lat, rel, None if disc is None else disc.ctypes.data, d, k, j))
    return d, k, j


# the reference's bundled topology (resource/topology.graphml.xml.xz, data file
# copied byte for byte): workload input for the configs on it
BUNDLED = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "topology.graphml.xml.xz")
# the one-vertex topology embedded in configs[0]'s example config
# (resource/examples/shadow.config.xml:2-23: 50 ms self-loop, packet loss 0.01)
C1_EMBEDDED = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "c1_topology.graphml")
