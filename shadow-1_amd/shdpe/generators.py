"""Synthetic topologies for the BASELINE.json configs.

All generators are seeded and deterministic.  Every vertex gets a self-loop:
the reference fold for target == source looks up edge (s,s)
(``topology.c:1469-1488``) and fails without it (SURVEY.md finding 4).

* C1  shipped ``resource/topology.graphml.xml.xz`` (fixture in tests/golden)
* C2  ``rgg(10_000, seed=1)``                 -- sparse, delta-stepping kernel
* C3  ``dense(20_000, seed=3)``               -- complete (a) / minus one edge (b)
* C4  ``power_law(100_000, m=3, seed=4)``     -- 16,384 attached (seed 5)
* C5  ``power_law(250_000, m=2, seed=6)``     -- 65,536 attached
"""
from __future__ import annotations

import numpy as np

from .graph import Topology


def _components(n, a, b):
    import scipy.sparse as sp
    from scipy.sparse.csgraph import connected_components
    g = sp.coo_matrix((np.ones(len(a)), (a, b)), shape=(n, n))
    return connected_components(g, directed=False)


def rgg(n: int = 10_000, seed: int = 1, mean_degree: float = 10.0,
        quantum: float = 0.0) -> Topology:
    """Random geometric graph in the unit square.

    radius r = sqrt(mean_degree / (pi n)); components are joined to the giant
    component by their nearest pair; latency = 1 + 300 * euclid ms; edge loss
    U[0, 0.01]; vertex loss 0.0; self-loop latency U[0.5, 2].  ``quantum`` > 0
    rounds latencies to multiples of it (tie-stress variant).
    """
    from scipy.spatial import cKDTree
    rng = np.random.default_rng(seed)
    pts = rng.random((n, 2))
    r = np.sqrt(mean_degree / (np.pi * n))
    tree = cKDTree(pts)
    pairs = tree.query_pairs(r, output_type="ndarray")
    a, b = pairs[:, 0].astype(np.int64), pairs[:, 1].astype(np.int64)
    ncomp, labels = _components(n, a, b)
    if ncomp > 1:
        giant = np.bincount(labels).argmax()
        gidx = np.flatnonzero(labels == giant)
        gtree = cKDTree(pts[gidx])
        extra_a, extra_b = [], []
        for c in range(ncomp):
            if c == giant:
                continue
            members = np.flatnonzero(labels == c)
            d, j = gtree.query(pts[members])
            k = int(np.argmin(d))
            extra_a.append(int(members[k]))
            extra_b.append(int(gidx[j[k]]))
        a = np.concatenate([a, np.array(extra_a, dtype=np.int64)])
        b = np.concatenate([b, np.array(extra_b, dtype=np.int64)])
    lo, hi = np.minimum(a, b), np.maximum(a, b)
    order = np.lexsort((hi, lo))
    lo, hi = lo[order], hi[order]
    euclid = np.sqrt(((pts[lo] - pts[hi]) ** 2).sum(axis=1))
    lat = 1.0 + 300.0 * euclid
    loss = rng.uniform(0.0, 0.01, size=lat.shape[0])
    self_lat = rng.uniform(0.5, 2.0, size=n)
    self_loss = rng.uniform(0.0, 0.01, size=n)
    src = np.concatenate([lo, np.arange(n)])
    dst = np.concatenate([hi, np.arange(n)])
    latency = np.concatenate([lat, self_lat])
    if quantum > 0:
        latency = np.maximum(np.round(latency / quantum), 1.0) * quantum
    top = Topology(n=n, directed=False, src=src, dst=dst, latency=latency,
                   loss=np.concatenate([loss, self_loss]), vloss=np.zeros(n),
                   name=f"rgg{n}_s{seed}" + (f"_q{quantum}" if quantum else ""))
    return top


def power_law(n: int = 100_000, m: int = 3, seed: int = 4, quantum: float = 0.0) -> Topology:
    """Barabasi-Albert preferential attachment.

    latency lognormal(ln 20, 0.7) ms, edge loss U[0, 0.02], self-loops.
    """
    rng = np.random.default_rng(seed)
    src_l, dst_l = [], []
    targets = list(range(m))
    repeated: list = []
    for source in range(m, n):
        src_l.extend([source] * m)
        dst_l.extend(targets)
        repeated.extend(targets)
        repeated.extend([source] * m)
        chosen = set()
        while len(chosen) < m:
            chosen.add(repeated[int(rng.integers(len(repeated)))])
        targets = sorted(chosen)
    a = np.array(src_l, dtype=np.int64)
    b = np.array(dst_l, dtype=np.int64)
    lat = rng.lognormal(np.log(20.0), 0.7, size=a.shape[0])
    loss = rng.uniform(0.0, 0.02, size=a.shape[0])
    self_lat = rng.lognormal(np.log(20.0), 0.7, size=n)
    self_loss = rng.uniform(0.0, 0.02, size=n)
    latency = np.concatenate([lat, self_lat])
    if quantum > 0:
        latency = np.maximum(np.round(latency / quantum), 1.0) * quantum
    return Topology(n=n, directed=False, src=np.concatenate([a, np.arange(n)]),
                    dst=np.concatenate([b, np.arange(n)]), latency=latency,
                    loss=np.concatenate([loss, self_loss]), vloss=np.zeros(n),
                    name=f"ba{n}_m{m}_s{seed}" + (f"_q{quantum}" if quantum else ""))


def _triu_pairs(n: int):
    """np.triu_indices(n, k=1) (row-major pairs i < j) as int32, without the
    n x n mask (C3: 2e8 pairs)."""
    cnt = np.arange(n - 1, 0, -1, dtype=np.int64)              # row i has n-1-i pairs
    iu = np.repeat(np.arange(n - 1, dtype=np.int32), cnt)
    start = np.concatenate([[0], np.cumsum(cnt)[:-1]])
    ju = np.arange(iu.shape[0], dtype=np.int64)
    ju -= np.repeat(start - np.arange(1, n, dtype=np.int64), cnt)
    return iu, ju.astype(np.int32)


def dense(n: int = 20_000, seed: int = 3, drop_edge: bool = False, quantum: float = 0.0) -> Topology:
    """Complete graph + self-loops; ``drop_edge`` removes
    one non-loop edge so ``_topology_isComplete`` is FALSE (C3b); ``quantum``
    rounds latencies to its multiples (0.005 ms: the tie-stress variant)."""
    rng = np.random.default_rng(seed)
    iu, ju = _triu_pairs(n)
    lat = np.clip(rng.lognormal(np.log(60.0), 0.8, size=iu.shape[0]), 1.0, 2000.0)
    if quantum > 0:
        lat = np.maximum(np.round(lat / quantum), 1.0) * quantum
    if drop_edge:
        k = int(rng.integers(iu.shape[0]))
        keep = np.ones(iu.shape[0], dtype=bool)
        keep[k] = False
        iu, ju, lat = iu[keep], ju[keep], lat[keep]
    self_lat = np.clip(rng.lognormal(np.log(60.0), 0.8, size=n), 1.0, 2000.0)
    if quantum > 0:
        self_lat = np.maximum(np.round(self_lat / quantum), 1.0) * quantum
    src = np.concatenate([iu, np.arange(n)])
    dst = np.concatenate([ju, np.arange(n)])
    latency = np.concatenate([lat, self_lat])
    return Topology(n=n, directed=False, src=src, dst=dst, latency=latency,
                    loss=np.full(latency.shape[0], 0.005), vloss=np.zeros(n),
                    name=f"dense{n}_s{seed}" + ("_minus1" if drop_edge else "") +
                    (f"_q{quantum}" if quantum > 0 else ""))


def random_sparse(n: int, avg_deg: float, seed: int, directed: bool = False,
                  quantum: float = 0.0, vloss: bool = False, self_loops: bool = True,
                  lat_lo: float = 1.0, lat_hi: float = 100.0) -> Topology:
    """Small connected random graphs for parity tests (ring + random chords)."""
    rng = np.random.default_rng(seed)
    perm = rng.permutation(n)
    a = [perm[i] for i in range(n - 1)]
    b = [perm[i + 1] for i in range(n - 1)]
    if directed and n > 1:
        a.append(perm[n - 1]); b.append(perm[0])          # strongly connected ring
    extra = max(0, int(n * avg_deg / 2) - len(a))
    ea = rng.integers(0, n, size=extra)
    eb = rng.integers(0, n, size=extra)
    seen = set()
    src, dst = [], []
    for x, y in zip(list(a) + list(ea), list(b) + list(eb)):
        x, y = int(x), int(y)
        if x == y:
            continue
        key = (x, y) if directed else (min(x, y), max(x, y))
        if key in seen:
            continue
        seen.add(key)
        src.append(x); dst.append(y)
    m = len(src)
    lat = rng.uniform(lat_lo, lat_hi, size=m)
    if self_loops:
        src += list(range(n)); dst += list(range(n))
        lat = np.concatenate([lat, rng.uniform(lat_lo, lat_hi, size=n)])
    if quantum > 0:
        lat = np.maximum(np.round(lat / quantum), 1.0) * quantum
    loss = rng.uniform(0.0, 0.05, size=len(src))
    vl = None
    if vloss:
        vl = rng.uniform(0.0, 0.05, size=n)
        vl[rng.random(n) < 0.2] = np.nan                   # some absent values
    return Topology(n=n, directed=directed, src=np.array(src), dst=np.array(dst),
                    latency=lat, loss=loss, vloss=vl, name=f"rand{n}_{seed}")


def minus_one_edge(top: Topology, seed: int = 0) -> Topology:
    """Remove one non-loop edge (forces isComplete=FALSE -> Dijkstra path)."""
    rng = np.random.default_rng(seed)
    cand = np.flatnonzero(top.src != top.dst)
    k = int(cand[rng.integers(cand.shape[0])])
    keep = np.ones(top.m, dtype=bool)
    keep[k] = False
    return Topology(n=top.n, directed=top.directed, src=top.src[keep], dst=top.dst[keep],
                    latency=top.latency[keep], loss=top.loss[keep], vloss=top.vloss,
                    ids=top.ids, prefers_direct=top.prefers_direct,
                    name=top.name + "_minus1")


def with_slower_newest_edges(top: Topology, frac: float, seed: int) -> Topology:
    """A multigraph where many groups' NEWEST parallel edge (igraph_get_eid's,
    the one the reference folds, topology.c:1488-1498) is SLOWER than an older
    one: copies of a fraction of the non-loop edges appended after the
    originals, half of them slower (x1.1-2.5), half faster, some groups of
    three; the reported latency is then the fold of the newest edges'
    latencies along the Dijkstra path, not the distance."""
    rng = np.random.default_rng(seed)
    cand = np.flatnonzero(top.src != top.dst)
    pick = rng.choice(cand, size=max(1, int(frac * cand.shape[0])), replace=False)
    src, dst, lat, loss = [top.src], [top.dst], [top.latency], [top.loss]
    for rep in range(2):
        sel = pick if rep == 0 else pick[rng.random(pick.shape[0]) < 0.3]
        slower = rng.random(sel.shape[0]) < 0.5
        l = top.latency[sel] * np.where(slower, rng.uniform(1.1, 2.5, sel.shape[0]),
                                        rng.uniform(0.4, 0.95, sel.shape[0]))
        if not top.directed:
            flip = rng.random(sel.shape[0]) < 0.5
            src.append(np.where(flip, top.dst[sel], top.src[sel]))
            dst.append(np.where(flip, top.src[sel], top.dst[sel]))
        else:
            src.append(top.src[sel]); dst.append(top.dst[sel])
        lat.append(l); loss.append(rng.uniform(0.0, 0.05, size=sel.shape[0]))
    return Topology(n=top.n, directed=top.directed, src=np.concatenate(src), dst=np.concatenate(dst),
                    latency=np.concatenate(lat), loss=np.concatenate(loss), vloss=top.vloss,
                    name=top.name + "_slow_newest")


def with_parallel_edges(top: Topology, frac: float, seed: int, consistent: bool = True,
                        loops: bool = True) -> Topology:
    """A multigraph: parallel copies of a fraction of the edges (and of the
    self-loops) appended after the originals, so each copy is the NEWEST edge
    of its group -- the one igraph_get_eid returns (oracle orc_get_eid).  With
    `consistent` every copy is also a fastest edge of its group (equal latency
    with another loss, or faster); otherwise one copy is slower than the edge
    it duplicates (see with_slower_newest_edges)."""
    rng = np.random.default_rng(seed)
    cand = np.flatnonzero(top.src != top.dst)
    if loops:
        cand = np.concatenate([cand, np.flatnonzero(top.src == top.dst)])
    pick = rng.choice(cand, size=max(1, int(frac * cand.shape[0])), replace=False)
    src, dst = [top.src], [top.dst]
    lat, loss = [top.latency], [top.loss]
    cur = {}
    for rep in range(2):                        # some groups get two copies
        sel = pick if rep == 0 else pick[rng.random(pick.shape[0]) < 0.3]
        l = np.array([cur.get(int(k), top.latency[k]) for k in sel])
        faster = rng.random(sel.shape[0]) < 0.5
        l = np.where(faster, l * rng.uniform(0.5, 1.0, size=sel.shape[0]), l)
        for k, x in zip(sel, l):
            cur[int(k)] = float(x)
        src.append(top.src[sel]); dst.append(top.dst[sel])
        # undirected copies sometimes list the endpoints the other way round
        if not top.directed:
            flip = rng.random(sel.shape[0]) < 0.5
            src[-1], dst[-1] = np.where(flip, top.dst[sel], top.src[sel]), np.where(flip, top.src[sel], top.dst[sel])
        lat.append(l); loss.append(rng.uniform(0.0, 0.05, size=sel.shape[0]))
    lat = np.concatenate(lat)
    if not consistent:
        lat[top.m] = top.latency[pick[0]] * 1.5   # the newest copy of pick[0] is slower
        if top.m + pick.shape[0] < lat.shape[0]:
            keep = np.ones(lat.shape[0], bool)
            keep[top.m + pick.shape[0]:] = False   # no second copies: pick[0]'s slow copy stays newest
            return Topology(n=top.n, directed=top.directed, src=np.concatenate(src)[keep],
                            dst=np.concatenate(dst)[keep], latency=lat[keep],
                            loss=np.concatenate(loss)[keep], vloss=top.vloss, name=top.name + "_multi_bad")
    return Topology(n=top.n, directed=top.directed, src=np.concatenate(src), dst=np.concatenate(dst),
                    latency=lat, loss=np.concatenate(loss), vloss=top.vloss,
                    name=top.name + ("_multi" if consistent else "_multi_bad"))


def with_parallel_loops(top: Topology, frac: float, seed: int) -> Topology:
    """Extra self-loops on a fraction of the looped vertices, one or two
    each, appended (newest), with latencies below, equal to or above the
    existing loop's: any order is legal (a loop never changes a distance; the
    (s, s) fold takes the newest loop, the self path the newest of minimum
    latency)."""
    rng = np.random.default_rng(seed)
    loops = np.flatnonzero(top.src == top.dst)
    pick = rng.choice(loops, size=max(1, int(frac * loops.shape[0])), replace=False)
    sel = np.concatenate([pick, pick[rng.random(pick.shape[0]) < 0.4]])
    f = rng.choice([0.5, 1.0, 1.0, 2.0], size=sel.shape[0])
    return Topology(n=top.n, directed=top.directed, src=np.concatenate([top.src, top.src[sel]]),
                    dst=np.concatenate([top.dst, top.dst[sel]]),
                    latency=np.concatenate([top.latency, top.latency[sel] * f]),
                    loss=np.concatenate([top.loss, rng.uniform(0.0, 0.05, size=sel.shape[0])]),
                    vloss=top.vloss, name=top.name + "_loops")


def sample_attached(n: int, k: int, seed: int) -> np.ndarray:
    """Attached vertices (``verticesWithAttachedHosts``), sorted."""
    if k >= n:
        return np.arange(n, dtype=np.int32)
    rng = np.random.default_rng(seed)
    return np.sort(rng.choice(n, size=k, replace=False)).astype(np.int32)


CONFIGS = {
    "c2": dict(desc="RGG n=10k, all 10k sources (BASELINE.json configs[1])"),
    "c4": dict(desc="BA n=100k m=3, 16,384 attached (configs[3], north_star target)"),
    "c4q": dict(desc="C4 with latencies rounded to 0.005 ms (tie stress, SURVEY.md 8d)"),
    "c2q": dict(desc="C2 with latencies rounded to 0.005 ms (tie stress, SURVEY.md 8d)"),
    "c3a": dict(desc="dense n=20k complete (configs[2], direct rows)"),
    "c3b": dict(desc="dense n=20k minus one edge (configs[2], min-plus)"),
    "c3bq": dict(desc="C3b with latencies rounded to 0.005 ms (dense tie stress, SURVEY.md 8d)"),
    "c5": dict(desc="BA n=250k m=2, 65,536 attached (configs[4])"),
    "c5q": dict(desc="C5 with latencies rounded to 0.005 ms (tie stress, SURVEY.md 8d)"),
}


def make_config(name: str):
    """Return (topology, attached) for a named config.

    c1   shipped topology (complete -> direct rows), 1 host per vertex
    c1m  shipped topology minus one edge (Dijkstra semantics, tie stress)
    c2   RGG 10k, all sources        c2q  same, latencies rounded to 0.005
    c3a  dense 20k complete           c3b  dense 20k minus one edge
    c3bq c3b, latencies rounded to 0.005 (SHDPE_C3_N overrides n for all three)
    c4   BA 100k, 16,384 attached     c4q  same, latencies rounded to 0.005
    c5   BA 250k, 65,536 attached     c5q  same, latencies rounded to 0.005
    """
    if name in ("c1", "c1m"):
        import os
        from .graph import Topology
        here = os.path.dirname(os.path.abspath(__file__))
        top = Topology.load_npz(os.path.join(here, "..", "..", "tests", "golden",
                                             "shipped_topology.npz"), name="shipped")
        if name == "c1m":
            top = minus_one_edge(top, seed=3)
        return top, np.arange(top.n, dtype=np.int32)
    if name in ("c3a", "c3b", "c3bq"):
        n = int(__import__("os").environ.get("SHDPE_C3_N", "20000"))
        top = dense(n, seed=3, drop_edge=(name != "c3a"), quantum=0.005 if name == "c3bq" else 0.0)
        return top, np.arange(top.n, dtype=np.int32)
    if name == "c2":
        top = rgg(10_000, seed=1)
        return top, np.arange(top.n, dtype=np.int32)
    if name == "c2q":
        top = rgg(10_000, seed=1, quantum=0.005)
        return top, np.arange(top.n, dtype=np.int32)
    if name in ("c4", "c4q"):
        top = power_law(100_000, m=3, seed=4, quantum=0.005 if name == "c4q" else 0.0)
        return top, sample_attached(top.n, 16_384, seed=5)
    if name in ("c5", "c5q"):
        top = power_law(250_000, m=2, seed=6, quantum=0.005 if name == "c5q" else 0.0)
        return top, sample_attached(top.n, 65_536, seed=7)
    raise KeyError(name)
