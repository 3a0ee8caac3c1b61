"""ctypes wrapper for the CPU oracle (oracle/pe_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, always as the checker / CPU baseline.  The
product path (shadow-1_amd/) never imports this module.

Parity pinning status: see DESIGN.md §"Oracle".  Direct-edge semantics are
pinned by the shipped topology and the reference's 1-vertex test configs;
Dijkstra distances and (tie-free) paths are pinned against scipy's
independent Dijkstra; igraph's equal-distance pop order is
"igraph-0.7.1-reconstructed" (igraph is absent here) -- parity unpinned for
that one aspect.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "_build", "libpe_oracle.so")

F_OK, F_UNREACHABLE, F_NOEDGE, F_ZEROLAT = 0, 1, 2, 4

_i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB


def _load():
    if not os.path.exists(_LIB):
        build()
    lib = C.CDLL(_LIB)
    vp = C.c_void_p
    lib.orc_graph_new.restype = vp
    lib.orc_graph_new.argtypes = [C.c_int32, C.c_int64, C.c_int32, vp, vp, vp, vp, vp]
    lib.orc_graph_free.argtypes = [vp]
    lib.orc_is_complete.argtypes = [vp]
    lib.orc_is_complete.restype = C.c_int32
    lib.orc_get_eid.argtypes = [vp, C.c_int32, C.c_int32]
    lib.orc_get_eid.restype = C.c_int64
    lib.orc_dijkstra_row.argtypes = [vp, C.c_int32, vp, C.c_int32, vp, vp, vp, vp, vp]
    lib.orc_dijkstra_row.restype = C.c_int32
    lib.orc_dijkstra_raw.argtypes = [vp, C.c_int32, vp, C.c_int32, vp, vp, vp, vp]
    lib.orc_dijkstra_raw.restype = C.c_int32
    lib.orc_direct_path.argtypes = [vp, C.c_int32, C.c_int32, vp, vp]
    lib.orc_direct_path.restype = C.c_int32
    lib.orc_self_path.argtypes = [vp, C.c_int32, vp, vp]
    lib.orc_self_path.restype = C.c_int32
    lib.orc_rows_parallel.argtypes = [vp, vp, C.c_int32, vp, C.c_int32, C.c_int32,
                                      vp, vp, vp, vp, vp]
    lib.orc_rows_parallel.restype = C.c_int32
    lib.orc_topology_new.restype = vp
    lib.orc_topology_new.argtypes = [vp, vp, C.c_int32, C.c_int32]
    lib.orc_topology_free.argtypes = [vp]
    for fn in ("orc_topology_get_latency", "orc_topology_get_reliability"):
        getattr(lib, fn).argtypes = [vp, C.c_int32, C.c_int32]
        getattr(lib, fn).restype = C.c_double
    for fn in ("orc_topology_is_routable", "orc_topology_increment_packet_counter"):
        getattr(lib, fn).argtypes = [vp, C.c_int32, C.c_int32]
        getattr(lib, fn).restype = C.c_int32
    lib.orc_topology_cached.argtypes = [vp, C.c_int32, C.c_int32, vp, vp, vp, vp]
    lib.orc_topology_cached.restype = C.c_int32
    lib.orc_topology_min_latency.argtypes = [vp]
    lib.orc_topology_min_latency.restype = C.c_double
    for fn in ("orc_topology_rows_computed", "orc_topology_self_paths_computed",
               "orc_topology_cache_size"):
        getattr(lib, fn).argtypes = [vp]
        getattr(lib, fn).restype = C.c_int64
    lib.orc_bellman_rows.argtypes = [vp, vp, C.c_int32, C.c_int32, vp]
    lib.orc_bellman_rows.restype = C.c_int32
    lib.orc_selftest_vector_order.argtypes = [C.c_int64, C.c_int32, C.c_uint64]
    lib.orc_selftest_vector_order.restype = C.c_int32
    return lib


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = _load()
    return _lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


class OracleGraph:
    """igraph-0.7.1-faithful graph + Dijkstra + topology.c fold (CPU)."""

    def __init__(self, top):
        L = lib()
        self.top = top
        self._keep = [top.src, top.dst, top.latency, top.loss, top.vloss]
        self.h = L.orc_graph_new(top.n, top.m, int(top.directed), _p(top.src), _p(top.dst),
                                 _p(top.latency), _p(top.loss), _p(top.vloss))
        if not self.h:
            raise ValueError("orc_graph_new failed")
        self.n = top.n

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.orc_graph_free(self.h)
            self.h = None

    def is_complete(self) -> bool:
        return bool(lib().orc_is_complete(self.h))

    def get_eid(self, a, b) -> int:
        return int(lib().orc_get_eid(self.h, a, b))

    def row(self, src: int, targets):
        t = np.ascontiguousarray(targets, dtype=np.int32)
        T = t.shape[0]
        lat = np.empty(T); rel = np.empty(T)
        hops = np.empty(T, np.int32); pred = np.empty(T, np.int32)
        flags = np.empty(T, np.uint8)
        rc = lib().orc_dijkstra_row(self.h, int(src), _p(t), T, _p(lat), _p(rel), _p(hops),
                                    _p(pred), _p(flags))
        if rc:
            raise ValueError("orc_dijkstra_row failed")
        return dict(lat=lat, rel=rel, hops=hops, pred=pred, flags=flags)

    def raw(self, src: int, targets):
        t = np.ascontiguousarray(targets, dtype=np.int32)
        dist = np.empty(self.n); par = np.empty(self.n, np.int64)
        order = np.empty(self.n, np.int32); popped = C.c_int32(0)
        rc = lib().orc_dijkstra_raw(self.h, int(src), _p(t), t.shape[0], _p(dist), _p(par),
                                    _p(order), C.byref(popped))
        if rc:
            raise ValueError("orc_dijkstra_raw failed")
        return dist, par, order[:popped.value]

    def rows(self, sources, targets, threads: int = 1):
        s = np.ascontiguousarray(sources, dtype=np.int32)
        t = np.ascontiguousarray(targets, dtype=np.int32)
        S, T = s.shape[0], t.shape[0]
        lat = np.empty((S, T)); rel = np.empty((S, T))
        hops = np.empty((S, T), np.int32); pred = np.empty((S, T), np.int32)
        flags = np.empty((S, T), np.uint8)
        rc = lib().orc_rows_parallel(self.h, _p(s), S, _p(t), T, int(threads), _p(lat),
                                     _p(rel), _p(hops), _p(pred), _p(flags))
        if rc:
            raise ValueError("orc_rows_parallel failed")
        return dict(lat=lat, rel=rel, hops=hops, pred=pred, flags=flags)

    def bellman_violations(self, sources, lat_rows, targets, threads: int = 1):
        """Checker: per row, arcs (u, v) whose relaxation would still shorten
        the row (0 for a shortest-path row).  lat_rows[r][j] = row r's latency
        to targets[j], which must cover every vertex; the source's own entry
        (the self-loop path) is replaced by 0."""
        t = np.asarray(targets)
        if np.unique(t).shape[0] != self.n or t.shape[0] != self.n:
            raise ValueError("bellman_violations needs rows over all vertices")
        R = len(sources)
        dT = np.empty((self.n, R))
        dT[t, :] = np.asarray(lat_rows, dtype=np.float64).T
        dT[np.asarray(sources), np.arange(R)] = 0.0
        dT = np.ascontiguousarray(dT)
        viol = np.zeros(R, np.int64)
        if lib().orc_bellman_rows(self.h, _p(dT), R, int(threads), _p(viol)):
            raise ValueError("orc_bellman_rows failed")
        return viol

    def direct(self, s, t):
        lat, rel = C.c_double(), C.c_double()
        rc = lib().orc_direct_path(self.h, int(s), int(t), C.byref(lat), C.byref(rel))
        return None if rc else (lat.value, rel.value)

    def self_path(self, v):
        lat, rel = C.c_double(), C.c_double()
        rc = lib().orc_self_path(self.h, int(v), C.byref(lat), C.byref(rel))
        return None if rc else (lat.value, rel.value)


class OracleTopology:
    """topology_getLatency/getReliability/isRoutable semantics with the
    path cache (topology.c:1284-1386, 1969-2092)."""

    def __init__(self, og: OracleGraph, attached, prefers_direct=False):
        self.og = og
        self._att = np.ascontiguousarray(attached, dtype=np.int32)
        self.h = lib().orc_topology_new(og.h, _p(self._att), self._att.shape[0],
                                        int(prefers_direct))
        if not self.h:
            raise ValueError("orc_topology_new failed")

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.orc_topology_free(self.h)
            self.h = None

    def get_latency(self, s, d):
        return lib().orc_topology_get_latency(self.h, int(s), int(d))

    def get_reliability(self, s, d):
        return lib().orc_topology_get_reliability(self.h, int(s), int(d))

    def is_routable(self, s, d):
        return bool(lib().orc_topology_is_routable(self.h, int(s), int(d)))

    def increment(self, s, d):
        return lib().orc_topology_increment_packet_counter(self.h, int(s), int(d))

    def cached(self, s, d):
        lat, rel = C.c_double(), C.c_double()
        isd, pc = C.c_int32(), C.c_int64()
        ok = lib().orc_topology_cached(self.h, int(s), int(d), C.byref(lat), C.byref(rel),
                                       C.byref(isd), C.byref(pc))
        return (lat.value, rel.value, bool(isd.value), pc.value) if ok else None

    @property
    def min_latency(self):
        return lib().orc_topology_min_latency(self.h)

    @property
    def rows_computed(self):
        return lib().orc_topology_rows_computed(self.h)

    @property
    def self_paths_computed(self):
        return lib().orc_topology_self_paths_computed(self.h)

    @property
    def cache_size(self):
        return lib().orc_topology_cache_size(self.h)
