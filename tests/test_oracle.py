"""CPU tests of the oracle (the checker) -- pinning it before trusting it.

Pins (DESIGN.md "Oracle"):
  * shipped topology + reference 1-vertex test topologies -> direct-path
    known answers computed independently from the input data;
  * scipy.sparse.csgraph.dijkstra (independent implementation) on tie-free
    graphs -> distances bit-exact, predecessors identical;
  * hand-derived igraph 2-wheap tie order;
  * committed golden rows (regression of the oracle itself).
"""
import json
import math
import os

import numpy as np
import pytest
import scipy.sparse as sp
from scipy.sparse.csgraph import dijkstra

from conftest import GOLDEN
from shdpe import generators as G
from shdpe.graph import Topology, read_graphml


def _og(oracle_mod, top):
    return oracle_mod.OracleGraph(top)


def _scipy(top):
    f, t = top.normalized_endpoints()
    nl = f != t
    A = sp.coo_matrix((top.latency[nl], (f[nl], t[nl])), shape=(top.n, top.n)).tocsr()
    return dijkstra(A, directed=top.directed, return_predecessors=True)


@pytest.mark.parametrize("seed,directed", [(1, False), (2, False), (3, True), (4, True)])
def test_oracle_matches_scipy_tiefree(oracle_mod, seed, directed):
    top = G.random_sparse(250, 5, seed=seed, directed=directed)
    og = _og(oracle_mod, top)
    D, P = _scipy(top)
    tg = np.arange(top.n, dtype=np.int32)
    for s in range(0, top.n, 3):
        r = og.row(s, tg)
        m = tg != s
        assert np.array_equal(r["lat"][m], D[s][m])             # left-fold dist, bit-exact
        assert np.array_equal(r["pred"][m], P[s][m])
        # hops = path length
        assert np.all(r["hops"][m] >= 1)
        assert not np.any(r["flags"])


def test_oracle_rgg_matches_scipy(oracle_mod):
    top = G.rgg(1500, seed=5)
    og = _og(oracle_mod, top)
    D, P = _scipy(top)
    tg = np.arange(top.n, dtype=np.int32)
    for s in (0, 7, 777, 1499):
        r = og.row(s, tg)
        m = tg != s
        assert np.array_equal(r["lat"][m], D[s][m])
        assert np.array_equal(r["pred"][m], P[s][m])


def test_shipped_topology_is_complete_and_direct(oracle_mod):
    top = Topology.load_npz(os.path.join(GOLDEN, "shipped_topology.npz"))
    assert (top.n, top.m) == (183, 16836)
    assert int((top.src == top.dst).sum()) == 183
    og = _og(oracle_mod, top)
    assert og.is_complete()
    # direct path for every pair, recomputed independently from the data:
    # lat = 0.0 + w, rel = ((1*a_s)*a_t)*(1-loss)   (topology.c:1887-1921)
    f, t = top.normalized_endpoints()
    W = {}
    for e in range(top.m):
        W[(int(f[e]), int(t[e]))] = (top.latency[e], 1.0 - top.loss[e])
    a = np.where(np.isnan(top.vloss), 1.0, 1.0 - top.vloss)
    rng = np.random.default_rng(0)
    for _ in range(2000):
        s, d = (int(x) for x in rng.integers(0, top.n, 2))
        lat, rel = og.direct(s, d)
        w, r = W[(max(s, d), min(s, d))]
        assert lat == 0.0 + w
        assert rel == ((1.0 * a[s]) * a[d]) * r


def test_minus_one_edge_is_incomplete(oracle_mod):
    top = Topology.load_npz(os.path.join(GOLDEN, "shipped_topology.npz"))
    m1 = G.minus_one_edge(top, seed=0)
    assert not _og(oracle_mod, m1).is_complete()
    # removing a self-loop instead also makes it incomplete (finding 4)
    keep = np.ones(top.m, bool)
    keep[np.flatnonzero(top.src == top.dst)[0]] = False
    nl = Topology(top.n, top.directed, top.src[keep], top.dst[keep], top.latency[keep],
                  top.loss[keep], top.vloss)
    assert not _og(oracle_mod, nl).is_complete()


def test_reference_test_topologies_known_answers(oracle_mod):
    cases = json.load(open(os.path.join(GOLDEN, "ref_test_topologies.json")))
    assert len(cases) >= 30
    for c in cases:
        vl = None if c["vloss"] is None else np.array(
            [math.nan if x is None else x for x in c["vloss"]])
        top = Topology(c["n"], c["directed"], np.array(c["src"]), np.array(c["dst"]),
                       np.array(c["latency"]), np.array(c["loss"]), vl)
        og = _og(oracle_mod, top)
        assert top.n == 1 and og.is_complete(), c["file"]
        lat, rel = og.direct(0, 0)
        a = 1.0 if vl is None or math.isnan(vl[0]) else 1.0 - vl[0]
        assert lat == c["latency"][0]
        assert rel == ((1.0 * a) * a) * (1.0 - c["loss"][0]), c["file"]


def test_igraph_2wheap_tie_order_hand_derived(oracle_mod):
    # 0-1 (1), 0-2 (1), 1-3 (1), 2-3 (1) + self-loops.  Popping 0 pushes 1 then
    # 2 with equal keys; shift_up swaps on equal keys (heap.c), so 2
    # pops before 1 and becomes parent of 3.
    src = np.array([0, 0, 1, 2, 0, 1, 2, 3])
    dst = np.array([1, 2, 3, 3, 0, 1, 2, 3])
    top = Topology(4, False, src, dst, np.array([1.0] * 4 + [5.0] * 4), np.zeros(8), None)
    og = _og(oracle_mod, top)
    dist, par, order = og.raw(0, np.arange(4, dtype=np.int32))
    assert list(order) == [0, 2, 1, 3]
    r = og.row(0, np.arange(4, dtype=np.int32))
    assert r["pred"][3] == 2 and r["hops"][3] == 2 and r["lat"][3] == 2.0
    # with vertex 1 and 2 swapped in id order the other one wins
    top2 = Topology(4, False, np.array([0, 0, 2, 1, 0, 1, 2, 3]), np.array([2, 1, 3, 3, 0, 1, 2, 3]),
                    top.latency, top.loss, None)
    r2 = _og(oracle_mod, top2).row(0, np.arange(4, dtype=np.int32))
    assert r2["pred"][3] == 2   # incidence order is by neighbour id, not edge id


def test_self_paths_and_missing_self_loop(oracle_mod):
    top = G.random_sparse(50, 4, seed=9)
    og = _og(oracle_mod, top)
    f, t = top.normalized_endpoints()
    for v in range(0, 50, 7):
        inc = [e for e in range(top.m) if f[e] == v or t[e] == v]
        ws = [top.latency[e] for e in inc]
        k = int(np.argmin(ws))
        lat, rel = og.self_path(v)
        assert lat == 2.0 * ws[k]
        r = 1.0 - top.loss[inc[k]]
        assert rel == r * r
    # Dijkstra row entry t==s uses the self-loop edge; without it -> NOEDGE
    keep = top.src != top.dst
    keep[np.flatnonzero(top.src == top.dst)[1:]] = True          # drop vertex 0's loop only
    nl = Topology(top.n, False, top.src[keep], top.dst[keep], top.latency[keep], top.loss[keep])
    r = _og(oracle_mod, nl).row(0, np.arange(50, dtype=np.int32))
    assert r["flags"][0] == oracle_mod.F_NOEDGE
    assert not np.any(r["flags"][1:])


def test_vertex_loss_nan_is_absent(oracle_mod):
    top = G.random_sparse(60, 4, seed=10, vloss=True)
    og = _og(oracle_mod, top)
    s = 3
    r = og.row(s, np.arange(60, dtype=np.int32))
    a = np.where(np.isnan(top.vloss), 1.0, 1.0 - top.vloss)
    # recompute one entry by walking the oracle's own path through preds
    for t in (10, 20, 30):
        path = [t]
        while path[-1] != s:
            path.append(int(r["pred"][path[-1]]))
        path = path[::-1]
        acc = (1.0 * a[s]) * a[t]
        for u, v in zip(path[:-1], path[1:]):
            e = og.get_eid(u, v)
            acc *= (1.0 - top.loss[e])
        assert acc == r["rel"][t]


def test_unreachable_directed(oracle_mod):
    # 0 -> 1 only: 1 cannot reach 0
    top = Topology(2, True, np.array([0, 0, 1]), np.array([1, 0, 1]), np.array([2.0, 1.0, 1.0]),
                   np.zeros(3))
    r = _og(oracle_mod, top).row(1, np.array([0, 1], np.int32))
    assert r["flags"][0] == oracle_mod.F_UNREACHABLE
    assert r["flags"][1] == 0 and r["lat"][1] == 1.0


def test_unreachable_target_keeps_row_success(oracle_mod):
    """topology.c:1815-1859: an empty igraph path (unreachable target) is
    skipped WITHOUT clearing isAllSuccess, so the lookup that triggered the
    row still succeeds; only a failed fold (missing (s,s) loop, :1857) fails
    it.  Directed 0 -> 1 -> 2 with 2 -> 1 only: from 1, vertex 0 is
    unreachable but (1,2) is found."""
    src = np.array([0, 1, 2, 0, 1, 2])
    dst = np.array([1, 2, 1, 0, 1, 2])
    top = Topology(3, True, src, dst, np.array([2.0, 3.0, 4.0, 1.0, 1.0, 1.0]), np.zeros(6))
    og = _og(oracle_mod, top)
    T = oracle_mod.OracleTopology(og, np.arange(3, dtype=np.int32))
    assert T.get_latency(1, 2) == 3.0              # row 1 has unreachable target 0
    assert T.rows_computed == 1
    assert T.cached(1, 0) is None                   # not stored (:1815)
    assert T.get_latency(1, 0) == -1.0              # the unreachable pair itself fails
    # a missing self-loop fails the fold of (s,s) -> the whole lookup fails (:1857)
    top2 = Topology(3, True, src[:5], dst[:5], np.array([2.0, 3.0, 4.0, 1.0, 1.0]), np.zeros(5))
    T2 = oracle_mod.OracleTopology(_og(oracle_mod, top2), np.arange(3, dtype=np.int32))
    assert T2.get_latency(2, 1) == -1.0            # row 2: (2,2) has no edge
    assert T2.cached(2, 1) is not None              # ... though (2,1) itself was stored


@pytest.mark.parametrize("name", ["rows_shipped_minus1", "rows_rand_tiefree", "rows_rand_quantized",
                                  "rows_rand_directed", "rows_rand_vloss", "rows_rgg2000",
                                  "rows_rgg2000_q"])
def test_golden_rows_regression(oracle_mod, name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    top = Topology(int(z["n"]), bool(z["directed"]), z["src"], z["dst"], z["latency"], z["loss"],
                   z["vloss"] if int(z["has_vloss"]) else None)
    og = _og(oracle_mod, top)
    res = og.rows(z["sources"], z["attached"], threads=4)
    for k in ("lat", "rel"):
        assert np.array_equal(res[k].view(np.int64), z[k].view(np.int64)), k
    for k in ("hops", "pred", "flags"):
        assert np.array_equal(res[k], z[k]), k


def test_topology_cache_semantics(oracle_mod):
    top = G.random_sparse(40, 4, seed=21)
    og = _og(oracle_mod, top)
    att = np.arange(0, 40, 2, dtype=np.int32)
    T = oracle_mod.OracleTopology(og, att)
    # (s,s) queried first -> self path (2*min edge), stored non-direct
    lat_ss = T.get_latency(4, 4)
    assert lat_ss == og.self_path(4)[0]
    # row for 4 computed later does not overwrite the cached (4,4)
    lat_48 = T.get_latency(4, 8)
    assert T.rows_computed == 1 and T.self_paths_computed == 1
    assert T.get_latency(4, 4) == lat_ss
    row = og.row(4, att)
    assert lat_48 == row["lat"][list(att).index(8)]
    # first-computed direction is cached for both directions
    assert T.get_latency(8, 4) == lat_48
    assert T.cached(8, 4) is None and T.cached(4, 8) is not None
    # row 8 computed on another miss keeps (4,8) entry
    T.get_latency(8, 10)
    assert T.rows_computed == 2
    assert T.cached(8, 4) is None
    # unattached vertex -> -1 (release-build error path)
    assert T.get_latency(4, 5) == -1.0
    assert T.increment(4, 8) == 0 and T.cached(4, 8)[3] == 1
    assert T.min_latency > 0


def test_topology_complete_graph_uses_direct(oracle_mod):
    top = Topology.load_npz(os.path.join(GOLDEN, "shipped_topology.npz"))
    og = _og(oracle_mod, top)
    att = np.arange(top.n, dtype=np.int32)
    T = oracle_mod.OracleTopology(og, att)
    for s, d in [(0, 5), (5, 0), (7, 7), (100, 3)]:
        lat = T.get_latency(s, d)
        assert lat == og.direct(s, d)[0] or lat == og.direct(d, s)[0]
    assert T.rows_computed == 0
    c = T.cached(0, 5)
    assert c is not None and c[2] is True


def test_topology_prefers_direct(oracle_mod):
    top = G.random_sparse(30, 4, seed=22)
    og = _og(oracle_mod, top)
    att = np.arange(30, dtype=np.int32)
    T = oracle_mod.OracleTopology(og, att, prefers_direct=True)
    f, t = top.normalized_endpoints()
    e = int(np.flatnonzero(f != t)[0])
    a, b = int(top.src[e]), int(top.dst[e])
    assert T.get_latency(a, b) == og.direct(a, b)[0]
    assert T.cached(a, b)[2] is True
    # a non-adjacent pair goes through a Dijkstra row; adjacent pairs of that
    # row are not stored as non-direct
    nonadj = [v for v in range(30) if v != a and og.get_eid(a, v) < 0][0]
    T.get_latency(a, nonadj)
    for v in range(30):
        if v != a and og.get_eid(a, v) >= 0 and v != b:
            assert T.cached(a, v) is None


def test_graphml_reader_doc_example():
    xml = open(os.path.join(os.path.dirname(__file__), "data", "doc_example.graphml")).read()
    top = read_graphml(xml)
    assert top.n == 1 and top.m == 1 and not top.directed
    assert top.latency[0] == 50.0 and top.loss[0] == 0.001 and top.vloss[0] == 0.0


@pytest.mark.parametrize("m,nodes", [(1000, 7), (50_000, 300), (200_000, 20_000)])
def test_vector_order_counting_form_matches_igraph_form(oracle_mod, m, nodes):
    """The oracle sorts huge edge lists (C3) with counting sorts; the order
    must be igraph_vector_order's exactly, parallel edges newest-first."""
    assert oracle_mod.lib().orc_selftest_vector_order(m, nodes, 12345) == 1
