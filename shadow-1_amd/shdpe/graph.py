"""Topology input model and GraphML reader (host side, harness only).

In Shadow the GraphML is parsed by igraph inside ``_topology_loadGraph``
(``src/main/routing/topology.c:371-399``) and stays in host C; the path engine
only receives the resulting edge list (ids in igraph order) through the C-ABI
(``include/shd_pathengine.h``).  Because igraph is not installable here, this
module reproduces the parts of igraph's GraphML import that define ids:

* vertex ids follow ``<node>`` document order;
* edge ids follow ``<edge>`` document order;
* numeric attributes are parsed as correctly rounded doubles; a missing value
  is NaN (``topology.c:330-370`` treats NaN as "absent").

Endpoint normalisation (undirected: ``from = max(a, b)``) is done by the
consumers exactly as ``igraph_add_edges`` does, so edges are kept here as
written in the file.
"""
from __future__ import annotations

import dataclasses
import io
import lzma
import math
import xml.etree.ElementTree as ET
from typing import Optional

import numpy as np

_NUMERIC = {"double", "float", "int", "long"}


@dataclasses.dataclass
class Topology:
    """A Shadow network topology as seen by the path engine.

    Attributes mirror the GraphML attributes Shadow reads on the hot path:
    edge ``latency`` / ``packetloss`` (``topology.c:1212-1246``, ``:402-444``)
    and optional vertex ``packetloss`` (``topology.c:1442-1462``).
    """

    n: int
    directed: bool
    src: np.ndarray            # int32[m], endpoints as written in the file
    dst: np.ndarray            # int32[m]
    latency: np.ndarray        # float64[m] (ms)
    loss: np.ndarray           # float64[m] in [0, 1]
    vloss: Optional[np.ndarray] = None   # float64[n]; None = attribute absent
    ids: Optional[list] = None           # vertex id strings
    prefers_direct: bool = False         # graph attr 'preferdirectpaths'
    name: str = "topology"

    @property
    def m(self) -> int:
        return int(self.src.shape[0])

    def __post_init__(self):
        self.src = np.ascontiguousarray(self.src, dtype=np.int32)
        self.dst = np.ascontiguousarray(self.dst, dtype=np.int32)
        self.latency = np.ascontiguousarray(self.latency, dtype=np.float64)
        self.loss = np.ascontiguousarray(self.loss, dtype=np.float64)
        if self.vloss is not None:
            self.vloss = np.ascontiguousarray(self.vloss, dtype=np.float64)

    # ------------------------------------------------------------------
    def validate(self) -> None:
        """Edge/vertex attribute checks of ``_topology_checkGraphEdgesHelperHook``
        (``topology.c:1041-1124``) and the vertex packetloss range check
        (``topology.c:956-970``)."""
        if self.m and (self.src.min() < 0 or self.dst.min() < 0 or
                       self.src.max() >= self.n or self.dst.max() >= self.n):
            raise ValueError("edge endpoint out of range")
        if np.any(~(self.latency > 0.0)):
            raise ValueError("edge latency must be > 0 and not NaN (topology.c:1070)")
        if np.any(~((self.loss >= 0.0) & (self.loss <= 1.0))):
            raise ValueError("edge packetloss must be in [0,1] (topology.c:1090)")
        if self.vloss is not None:
            v = self.vloss[~np.isnan(self.vloss)]
            if np.any((v < 0.0) | (v > 1.0)):
                raise ValueError("vertex packetloss must be in [0,1] (topology.c:961)")

    def normalized_endpoints(self):
        """(from, to) as igraph stores them (igraph_add_edges)."""
        if self.directed:
            return self.src.copy(), self.dst.copy()
        a, b = self.src, self.dst
        return np.maximum(a, b).astype(np.int32), np.minimum(a, b).astype(np.int32)

    def save_npz(self, path: str) -> None:
        np.savez_compressed(
            path, n=np.int64(self.n), directed=np.int8(self.directed),
            src=self.src, dst=self.dst, latency=self.latency, loss=self.loss,
            vloss=(self.vloss if self.vloss is not None else np.zeros(0)),
            has_vloss=np.int8(self.vloss is not None),
            prefers_direct=np.int8(self.prefers_direct),
            ids=np.array(self.ids if self.ids is not None else [], dtype=np.str_))

    @staticmethod
    def load_npz(path: str, name: str = "topology") -> "Topology":
        z = np.load(path, allow_pickle=False)
        ids = [str(x) for x in z["ids"]] or None
        return Topology(n=int(z["n"]), directed=bool(z["directed"]), src=z["src"],
                        dst=z["dst"], latency=z["latency"], loss=z["loss"],
                        vloss=(z["vloss"] if int(z["has_vloss"]) else None), ids=ids,
                        prefers_direct=bool(z["prefers_direct"]), name=name)


def _strip(tag: str) -> str:
    return tag.rsplit("}", 1)[-1]


def _parse_num(text: Optional[str]) -> float:
    if text is None:
        return math.nan
    t = text.strip()
    if not t:
        return math.nan
    try:
        return float(t)
    except ValueError:
        return math.nan


def read_graphml(source, name: str = "topology") -> Topology:
    """Read a Shadow GraphML topology (path, bytes, str, or .xz path)."""
    if isinstance(source, (bytes, bytearray)):
        data = bytes(source)
    elif isinstance(source, str) and source.lstrip().startswith("<"):
        data = source.encode()
    else:
        with open(source, "rb") as f:
            data = f.read()
        if str(source).endswith(".xz"):
            data = lzma.decompress(data)
    root = ET.parse(io.BytesIO(data)).getroot()
    keys = {}     # key id -> (for, name, type, default)
    for k in root:
        if _strip(k.tag) != "key":
            continue
        default = None
        for c in k:
            if _strip(c.tag) == "default":
                default = c.text
        keys[k.get("id")] = (k.get("for"), k.get("attr.name"), k.get("attr.type"), default)
    graph = next(c for c in root if _strip(c.tag) == "graph")
    directed = graph.get("edgedefault", "directed") == "directed"

    def defaults(kind):
        out = {}
        for kid, (f, an, at, d) in keys.items():
            if f == kind and d is not None:
                out[an] = _parse_num(d) if at in _NUMERIC else d
        return out

    gattrs = defaults("graph")
    for c in graph:
        if _strip(c.tag) == "data" and c.get("key") in keys:
            f, an, at, _ = keys[c.get("key")]
            if f == "graph":
                gattrs[an] = _parse_num(c.text) if at in _NUMERIC else (c.text or "")

    node_ids, vloss_list, id_index = [], [], {}
    has_vloss = any(f == "node" and an == "packetloss" for f, an, _, _ in keys.values())
    nd = defaults("node")
    ed = defaults("edge")
    edges = []
    for c in graph:
        tag = _strip(c.tag)
        if tag == "node":
            attrs = dict(nd)
            for d in c:
                if _strip(d.tag) == "data" and d.get("key") in keys:
                    f, an, at, _ = keys[d.get("key")]
                    attrs[an] = _parse_num(d.text) if at in _NUMERIC else (d.text or "")
            id_index[c.get("id")] = len(node_ids)
            node_ids.append(c.get("id"))
            vloss_list.append(attrs.get("packetloss", math.nan))
        elif tag == "edge":
            attrs = dict(ed)
            for d in c:
                if _strip(d.tag) == "data" and d.get("key") in keys:
                    f, an, at, _ = keys[d.get("key")]
                    attrs[an] = _parse_num(d.text) if at in _NUMERIC else (d.text or "")
            edges.append((c.get("source"), c.get("target"),
                          attrs.get("latency", math.nan), attrs.get("packetloss", math.nan)))
    src = np.array([id_index[e[0]] for e in edges], dtype=np.int32)
    dst = np.array([id_index[e[1]] for e in edges], dtype=np.int32)
    lat = np.array([e[2] for e in edges], dtype=np.float64)
    loss = np.array([e[3] for e in edges], dtype=np.float64)
    pdp = gattrs.get("preferdirectpaths")
    prefers = False
    if isinstance(pdp, str) and pdp:
        # topology.c:769-790: case-insensitive prefix match on true/yes/1
        low = pdp.lower()
        prefers = low.startswith("true") or low.startswith("yes") or low.startswith("1")
    return Topology(n=len(node_ids), directed=directed, src=src, dst=dst, latency=lat,
                    loss=loss, vloss=(np.array(vloss_list) if has_vloss else None),
                    ids=node_ids, prefers_direct=prefers, name=name)


def write_graphml(top: Topology) -> str:
    """Serialise a Topology as Shadow GraphML (used for fixtures/examples)."""
    out = ['<?xml version="1.0" encoding="utf-8"?>',
           '<graphml xmlns="http://graphml.graphdrawing.org/xmlns">',
           '  <key attr.name="packetloss" attr.type="double" for="edge" id="d1" />',
           '  <key attr.name="latency" attr.type="double" for="edge" id="d0" />']
    if top.vloss is not None:
        out.append('  <key attr.name="packetloss" attr.type="double" for="node" id="d2" />')
    if top.prefers_direct:
        out.append('  <key attr.name="preferdirectpaths" attr.type="string" for="graph" id="d3" />')
    out.append('  <graph edgedefault="%s">' % ("directed" if top.directed else "undirected"))
    if top.prefers_direct:
        out.append('    <data key="d3">true</data>')
    ids = top.ids or ["v%d" % i for i in range(top.n)]
    for i in range(top.n):
        if top.vloss is not None and not math.isnan(top.vloss[i]):
            out.append('    <node id="%s"><data key="d2">%r</data></node>' % (ids[i], float(top.vloss[i])))
        else:
            out.append('    <node id="%s"/>' % ids[i])
    for e in range(top.m):
        out.append('    <edge source="%s" target="%s"><data key="d0">%r</data>'
                   '<data key="d1">%r</data></edge>' % (ids[top.src[e]], ids[top.dst[e]],
                                                       float(top.latency[e]), float(top.loss[e])))
    out.append("  </graph>")
    out.append("</graphml>")
    return "\n".join(out)
