"""GPU parity: the HIP path (through the C-ABI) against the oracle.

Bar (BASELINE.json north_star): chosen paths (predecessor) and hop counts
bit-exact, latency and reliability bit-exact (the 1e-12 relative tolerance of
north_star is not needed: both sides fold in the reference order).
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from shdpe import generators as G
from shdpe.graph import Topology

pytestmark = pytest.mark.gpu

REL_TOL = 1e-12   # north_star tolerance; the asserts below are stricter (bit-exact)


@pytest.fixture(scope="module")
def E():
    from shdpe import engine
    engine.load_library()
    return engine


def _assert_rows_equal(got, exp, ctx=""):
    fails = (exp["flags"] & 0x03) != 0
    ok = ~fails
    assert np.array_equal(got["flags"] & 0x03, exp["flags"] & 0x03), ctx
    for k in ("lat", "rel"):
        g, e = got[k][ok], exp[k][ok]
        bad = np.flatnonzero(g.view(np.int64) != e.view(np.int64))
        assert bad.size == 0, f"{ctx} {k} first bad {bad[:5]} got {g[bad[:3]]} exp {e[bad[:3]]}"
        assert np.allclose(g, e, rtol=REL_TOL, atol=0)
    assert np.array_equal(got["hops"][ok], exp["hops"][ok]), ctx
    if got.get("pred") is not None:
        assert np.array_equal(got["pred"][ok], exp["pred"][ok]), ctx


def _check_engine(E, oracle_mod, top, att, sources=None, force=0, debug_flags=0):
    eng = E.Engine(top, att, force_mode=force, debug_flags=debug_flags)
    og = oracle_mod.OracleGraph(top)
    srcs = eng.attached if sources is None else np.asarray(sources, np.int32)
    eng.compute_rows(srcs)
    exp = og.rows(srcs, eng.attached, threads=8)
    for i, s in enumerate(srcs):
        g = eng.get_row(int(s))
        _assert_rows_equal(g, {k: v[i] for k, v in exp.items()}, f"row {s}")
    st = eng.stats()
    eng.close()
    if not os.environ.get("SHDPE_TIE_CORRUPT"):
        # the exact kernels' tie-slot cross-check never fires on a correct run
        assert st["rowsTieRepaired"] == 0, st
    return st


@pytest.mark.parametrize("name", ["rows_shipped_minus1", "rows_rand_tiefree", "rows_rand_quantized",
                                  "rows_rand_directed", "rows_rand_vloss", "rows_rgg2000",
                                  "rows_rgg2000_q"])
def test_golden_fixtures(E, name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    top = Topology(int(z["n"]), bool(z["directed"]), z["src"], z["dst"], z["latency"], z["loss"],
                   z["vloss"] if int(z["has_vloss"]) else None)
    eng = E.Engine(top, z["attached"])
    assert np.array_equal(eng.attached, z["attached"])
    eng.compute_rows(z["sources"])
    for i, s in enumerate(z["sources"]):
        _assert_rows_equal(eng.get_row(int(s)), {k: z[k][i] for k in
                                                 ("lat", "rel", "hops", "pred", "flags")},
                           f"{name} row {s}")
    eng.close()


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_random_tiefree(E, oracle_mod, seed):
    top = G.random_sparse(500, 5, seed=100 + seed)
    st = _check_engine(E, oracle_mod, top, np.arange(500))
    assert st["rowsExact"] == 0


def test_directed(E, oracle_mod):
    top = G.random_sparse(400, 4, seed=7, directed=True)
    _check_engine(E, oracle_mod, top, np.arange(400))


def test_vertex_loss(E, oracle_mod):
    top = G.random_sparse(400, 4, seed=8, vloss=True)
    _check_engine(E, oracle_mod, top, np.arange(0, 400, 3))


def test_quantized_ties_use_exact_kernel(E, oracle_mod):
    top = G.random_sparse(400, 6, seed=9, quantum=1.0)
    st = _check_engine(E, oracle_mod, top, np.arange(400))
    assert st["rowsExact"] > 0
    assert st["rowsTieEarly"] > 0      # k_sparse_rows tie export -> early stop


def test_forced_exact_kernel_all_rows(E, oracle_mod):
    top = G.random_sparse(300, 5, seed=10, quantum=2.0, directed=True)
    st = _check_engine(E, oracle_mod, top, np.arange(300), force=3)
    assert st["rowsExact"] == 300


def test_exact_kernel_heap_tail_in_global(E, oracle_mod, monkeypatch):
    """k_exact_rows with only 5 heap entries in LDS: the rest of the igraph
    2-way heap lives in the global slot (the split the large graphs use)."""
    monkeypatch.setenv("SHDPE_EXACT_HC", "5")
    top = G.random_sparse(300, 5, seed=11, quantum=2.0)
    st = _check_engine(E, oracle_mod, top, np.arange(0, 300, 3), force=3, debug_flags=E.DEBUG_ENV)
    assert st["rowsExact"] == 100


@pytest.mark.parametrize("n,hc", [(3000, 2100), (20000, 2400)])
def test_exact_kernel_small_lds_top(E, oracle_mod, monkeypatch, n, hc):
    """k_exact_rows with a small LDS top of the heap (hc of 2,100 / 2,400
    positions: most sift-downs, pushes and modifies reach the global tail) on
    quantised power-law graphs above the all-LDS size: every row bit-exact."""
    monkeypatch.setenv("SHDPE_EXACT_HC", str(hc))
    top = G.power_law(n, m=3, seed=21, quantum=0.5)
    att = G.sample_attached(n, 300, seed=5)
    st = _check_engine(E, oracle_mod, top, att, sources=att[:24], force=3, debug_flags=E.DEBUG_ENV)
    assert st["rowsExact"] == 24


def test_exact_kernel_large_graph_global_index(E, oracle_mod):
    """n > 24k: index2 in global memory, heap head in LDS, tail in global."""
    top = G.power_law(30_000, m=2, seed=12)
    att = G.sample_attached(top.n, 600, seed=4)
    st = _check_engine(E, oracle_mod, top, att, sources=att[:6], force=3)
    assert st["rowsExact"] == 6


def test_shipped_minus_one_edge_ties(E, oracle_mod):
    top = Topology.load_npz(os.path.join(GOLDEN, "shipped_topology.npz"))
    m1 = G.minus_one_edge(top, seed=3)
    st = _check_engine(E, oracle_mod, m1, np.arange(top.n))
    assert st["rowsExact"] > 0        # 0.005-quantised latencies -> equal-dist ties


def test_bulk_get_rows_matches_get_row(E):
    """shd_pe_get_rows (staged bulk D2H, several staging blocks) returns the
    same bytes as per-row shd_pe_get_row."""
    top = G.rgg(3000, seed=21)
    eng = E.Engine(top, np.arange(top.n))
    eng.compute_all()
    blk = eng.get_rows(5, 2990)        # 2990 rows x 3000 x 25 B = 224 MB > 2 x 64 MB staging
    pin = eng.pinned_rows(2990)        # shd_pe_host_alloc buffers: direct DMA, no staging
    eng.get_rows(5, 2990, out=pin)
    for k in ("lat", "rel", "hops", "pred", "flags"):
        assert np.array_equal(blk[k].view(np.uint8), pin[k].view(np.uint8)), k
    for i in (0, 1, 1337, 2989):
        one = eng.get_row(int(eng.attached[5 + i]))
        for k in ("lat", "rel", "hops", "pred", "flags"):
            assert np.array_equal(blk[k][i].view(np.uint8), one[k].view(np.uint8)), (i, k)
    with pytest.raises(E.EngineError):
        eng.get_rows(2990, 100)
    eng.close()


def test_partial_attached_and_unattached_source(E, oracle_mod):
    top = G.rgg(3000, seed=9)
    att = G.sample_attached(top.n, 700, seed=1)
    _check_engine(E, oracle_mod, top, att, sources=att[::7])
    eng = E.Engine(top, att)
    with pytest.raises(E.EngineError):
        eng.get_row(int(np.setdiff1d(np.arange(top.n), att)[0]))
    eng.close()


def test_power_law_hubs(E, oracle_mod):
    top = G.power_law(6000, m=3, seed=4)
    att = G.sample_attached(top.n, 1000, seed=2)
    _check_engine(E, oracle_mod, top, att, sources=att[::20])


def test_large_graph_hbm_layout(E, oracle_mod):
    top = G.power_law(60_000, m=2, seed=6)
    att = G.sample_attached(top.n, 2000, seed=3)
    _check_engine(E, oracle_mod, top, att, sources=att[::100])


def test_missing_self_loop_and_unreachable(E, oracle_mod):
    # directed 0->1->2, 2->0 plus 3 that only points in; vertex 1 has no loop
    src = np.array([0, 1, 2, 3, 0, 2, 3])
    dst = np.array([1, 2, 0, 0, 0, 2, 3])
    top = Topology(4, True, src, dst, np.array([1.0, 2.0, 3.0, 4.0, 0.5, 0.5, 0.5]), np.zeros(7))
    _check_engine(E, oracle_mod, top, np.arange(4))
    eng = E.Engine(top, np.arange(4))
    r = eng.get_row(1)
    assert r["flags"][1] & E.F_NOEDGE
    r0 = eng.get_row(0)
    assert r0["flags"][3] & E.F_UNREACHABLE
    eng.close()


def test_complete_graph_direct_rows(E, oracle_mod):
    top = Topology.load_npz(os.path.join(GOLDEN, "shipped_topology.npz"))
    og = oracle_mod.OracleGraph(top)
    eng = E.Engine(top, np.arange(top.n))
    assert eng.is_complete
    eng.compute_all()
    for s in (0, 17, 182):
        r = eng.get_row(s)
        assert np.all(r["flags"] == E.F_DIRECT)
        for t in range(top.n):
            lat, rel = og.direct(s, t)
            assert r["lat"][t] == lat and r["rel"][t] == rel
    assert eng.stats()["mode"] == 2
    eng.close()


def test_multigraph_newest_slower_small(E, oracle_mod):
    """The newest parallel edge (igraph_get_eid's, the one the reference
    folds, topology.c:1488-1498) slower than an older one: Dijkstra runs on
    the faster edge, the reported latency folds the newest one's -- row
    latency 2.0 over a distance of 1.0 (was rejected with EMULTI before
    round 5)."""
    top = Topology(3, False, np.array([0, 1, 0, 0, 1, 2]), np.array([1, 0, 0, 2, 1, 2]),
                   np.array([1.0, 2.0, 1.0, 1.0, 1.0, 1.0]), np.zeros(6))
    _check_engine(E, oracle_mod, top, np.arange(3))
    eng = E.Engine(top, np.arange(3))
    eng.compute_all()
    assert eng.get_row(0)["lat"][1] == 2.0
    eng.close()


@pytest.mark.parametrize("directed", [False, True], ids=["undirected", "directed"])
@pytest.mark.parametrize("quantum", [0.0, 10.0], ids=["tiefree", "quantised"])
@pytest.mark.parametrize("force", [0, 5], ids=["sparse", "batched"])
def test_multigraph_newest_slower_rows(E, oracle_mod, directed, quantum, force):
    """Multigraphs where half of the parallel groups' newest edge is the
    slower one (HostGraph::latFold): every row through the exact emulation
    with the folded-latency label, bit-exact against the oracle's igraph run
    over the unmerged edge list (n = 400: the all-LDS heap kernel)."""
    base = G.random_sparse(400, 5, seed=51 + int(directed), directed=directed, quantum=quantum, vloss=True)
    top = G.with_slower_newest_edges(base, 0.3, seed=9)
    st = _check_engine(E, oracle_mod, top, np.arange(0, 400, 3, dtype=np.int32), force=force)
    assert st["rowsExact"] > 0


@pytest.mark.parametrize("hc", [0, 64], ids=["lds_head", "global_tail"])
def test_multigraph_newest_slower_large(E, oracle_mod, monkeypatch, hc):
    """The same on n = 12,000 (k_exact_rows: the preferred-child-bit heap;
    with SHDPE_EXACT_HC=64 the heap lives almost wholly in the global tail)."""
    dbg = 0
    if hc:
        monkeypatch.setenv("SHDPE_EXACT_HC", str(hc))
        dbg = E.DEBUG_ENV
    top = G.with_slower_newest_edges(G.random_sparse(12000, 5, seed=61, quantum=10.0), 0.2, seed=10)
    _check_engine(E, oracle_mod, top, np.arange(0, 12000, 500, dtype=np.int32),
                  sources=np.arange(0, 12000, 1000, dtype=np.int32), debug_flags=dbg)


def test_multigraph_newest_slower_complete(E, oracle_mod):
    """A complete multigraph (direct rows, topology.c:1877-1927): the direct
    path reads igraph_get_eid's edge, the newest parallel one."""
    base = G.dense(40, seed=5)
    top = G.with_slower_newest_edges(base, 0.3, seed=11)
    og = oracle_mod.OracleGraph(top)
    eng = E.Engine(top, np.arange(top.n))
    assert eng.is_complete
    eng.compute_all()
    for s in range(top.n):
        r = eng.get_row(s)
        assert np.all(r["flags"] == E.F_DIRECT)
        for t in range(top.n):
            lat, rel = og.direct(s, t)
            assert r["lat"][t] == lat and r["rel"][t] == rel, (s, t)
    assert eng.stats()["mode"] == 2
    eng.close()


@pytest.mark.parametrize("directed", [False, True], ids=["undirected", "directed"])
@pytest.mark.parametrize("quantum", [0.0, 10.0], ids=["tiefree", "quantised"])
@pytest.mark.parametrize("force", [0, 5], ids=["sparse", "batched"])
def test_multigraph_rows(E, oracle_mod, directed, quantum, force):
    """Multigraphs (topology.c:417-420: igraph_get_eid picks the newest parallel
    edge for the fold; Dijkstra relaxes every parallel edge in incidence order,
    newest first): parallel copies of 30% of the edges and self-loops, each
    copy the newest of its group and a fastest one, some groups of three,
    vertex loss; every row bit-exact against the oracle's igraph-faithful
    run over the unmerged edge list, tie rows through the exact kernel."""
    base = G.random_sparse(400, 5, seed=41 + int(directed), directed=directed, quantum=quantum, vloss=True)
    top = G.with_parallel_edges(base, 0.3, seed=7)
    assert top.m > base.m + 100
    st = _check_engine(E, oracle_mod, top, np.arange(0, 400, 3, dtype=np.int32), force=force)
    if force == 5:
        assert st["mode"] == 1
    if quantum > 0:
        assert st["rowsExact"] > 0          # tie rows went through the igraph heap emulation


@pytest.mark.parametrize("directed", [False, True], ids=["undirected", "directed"])
@pytest.mark.parametrize("force", [0, 5], ids=["sparse", "batched"])
def test_parallel_self_loops_rows(E, oracle_mod, directed, force):
    """Several self-loops per vertex in any latency order (the newest may be
    the slowest): accepted; every row bit-exact against the oracle -- the
    (s, s) entry folds the newest loop (igraph_get_eid) -- and the direct
    (s, s) lookup agrees."""
    top = G.with_parallel_loops(G.random_sparse(300, 5, seed=51, directed=directed, vloss=True), 0.7, seed=3)
    loops = top.src == top.dst
    assert np.bincount(top.src[loops], minlength=top.n).max() >= 3
    att = np.arange(0, 300, 2, dtype=np.int32)
    _check_engine(E, oracle_mod, top, att, force=force)
    eng = E.Engine(top, att)
    og = oracle_mod.OracleGraph(top)
    for v in range(0, 300, 7):
        assert eng.direct_path(v, v) == og.direct(v, v), v
    eng.close()


def test_multigraph_complete_direct_rows(E, oracle_mod):
    """Complete multigraphs take the direct rows: every entry is the newest
    parallel edge's (latency, reliability), as _topology_lookupDirectPath
    reads it through igraph_get_eid (topology.c:1877-1927)."""
    top = G.with_parallel_edges(G.dense(60, seed=5), 0.3, seed=9)
    og = oracle_mod.OracleGraph(top)
    eng = E.Engine(top, np.arange(top.n, dtype=np.int32))
    assert eng.is_complete and og.is_complete()
    assert eng.is_complete_device() == 1
    eng.compute_all()
    for s in range(top.n):
        r = eng.get_row(s)
        assert np.all(r["flags"] == E.F_DIRECT)
        for t in range(top.n):
            lat, rel = og.direct(s, t)
            assert r["lat"][t] == lat and r["rel"][t] == rel, (s, t)
    eng.close()


def test_multigraph_counted_complete(E, oracle_mod):
    """_topology_isComplete counts incident EDGES (topology.c:450-552): a
    complete graph missing edge {a, b} but with a parallel copy of another
    edge at a and at b still counts as complete, so the reference serves
    direct paths and (a, b) has none.  The topology mirror matches the
    oracle's cache protocol on it, query for query."""
    d = G.dense(40, seed=6)
    a, b = 3, 17
    drop = ((d.src == a) & (d.dst == b)) | ((d.src == b) & (d.dst == a))
    keep = ~drop
    src = np.concatenate([d.src[keep], [a, b]])
    dst = np.concatenate([d.dst[keep], [5, 9]])
    lat_ab = [d.latency[keep][((d.src[keep] == x) & (d.dst[keep] == y)) | ((d.src[keep] == y) & (d.dst[keep] == x))][0]
              for x, y in ((a, 5), (b, 9))]
    top = Topology(d.n, False, src, dst, np.concatenate([d.latency[keep], lat_ab]),
                   np.concatenate([d.loss[keep], [0.01, 0.02]]), d.vloss)
    og = oracle_mod.OracleGraph(top)
    att = np.arange(top.n, dtype=np.int32)
    eng = E.Engine(top, att)
    assert og.is_complete() and eng.is_complete and eng.is_complete_device() == 1
    ref = oracle_mod.OracleTopology(og, att)
    shim = E.TopologyShim(eng)
    pairs = [(a, b), (b, a), (a, a), (a, 5), (5, a), (b, 9)]
    rng = np.random.default_rng(2)
    pairs += [tuple(int(x) for x in rng.integers(0, top.n, 2)) for _ in range(1500)]
    for s, t in pairs:
        x = (ref.get_latency(s, t), ref.get_reliability(s, t), ref.is_routable(s, t))
        y = (shim.get_latency(s, t), shim.get_reliability(s, t), shim.is_routable(s, t))
        assert x == y, (s, t, x, y)
    assert ref.cache_size == shim.cache_size
    shim.close()
    eng.close()


def test_invalid_latency_rejected(E):
    top = Topology(2, False, np.array([0, 0, 1]), np.array([1, 0, 1]), np.array([0.0, 1, 1]),
                   np.zeros(3))
    with pytest.raises(E.EngineError) as ei:
        E.Engine(top, np.arange(2))
    assert ei.value.code == E.EINVAL


def test_topology_shim_matches_oracle_cache(E, oracle_mod):
    top = G.random_sparse(200, 4, seed=31, vloss=True)
    att = np.arange(0, 200, 2, dtype=np.int32)
    for prefers in (False, True):
        og = oracle_mod.OracleGraph(top)
        ref = oracle_mod.OracleTopology(og, att, prefers_direct=prefers)
        eng = E.Engine(top, att)
        shim = E.TopologyShim(eng, prefers_direct=prefers)
        rng = np.random.default_rng(5)
        for _ in range(3000):
            s, d = (int(x) for x in rng.choice(att, 2))
            if rng.random() < 0.05:
                d = s
            a = (ref.get_latency(s, d), ref.get_reliability(s, d), ref.is_routable(s, d))
            b = (shim.get_latency(s, d), shim.get_reliability(s, d), shim.is_routable(s, d))
            assert a == b, (s, d, a, b)
            assert ref.increment(s, d) == shim.increment(s, d)
        assert ref.cache_size == shim.cache_size
        assert ref.min_latency == shim.min_latency
        for s in att[::5]:
            for d in att[::5]:
                assert ref.cached(int(s), int(d)) == shim.cached(int(s), int(d))
        shim.close()
        eng.close()


def test_topology_shim_complete_graph(E, oracle_mod):
    top = Topology.load_npz(os.path.join(GOLDEN, "shipped_topology.npz"))
    att = np.arange(top.n, dtype=np.int32)
    ref = oracle_mod.OracleTopology(oracle_mod.OracleGraph(top), att)
    eng = E.Engine(top, att)
    shim = E.TopologyShim(eng)
    rng = np.random.default_rng(1)
    for _ in range(2000):
        s, d = (int(x) for x in rng.integers(0, top.n, 2))
        assert ref.get_latency(s, d) == shim.get_latency(s, d)
        assert ref.get_reliability(s, d) == shim.get_reliability(s, d)
    assert ref.cache_size == shim.cache_size
    shim.close()
    eng.close()


def test_c2_full_table_properties(E, oracle_mod):
    """BASELINE config C2 at full size: sampled rows bit-exact vs the oracle,
    every row satisfies the size-independent invariants."""
    top, att = G.make_config("c2")
    eng = E.Engine(top, att)
    eng.compute_all()
    st = eng.stats()
    assert st["rowsComputed"] == 10_000
    og = oracle_mod.OracleGraph(top)
    rng = np.random.default_rng(11)
    sample = rng.choice(att, 24, replace=False)
    exp = og.rows(sample, att, threads=8)
    for i, s in enumerate(sample):
        _assert_rows_equal(eng.get_row(int(s)), {k: v[i] for k, v in exp.items()}, f"c2 row {s}")
    # invariants on a sweep of rows: Bellman consistency with the chosen
    # predecessor (lat[t] == lat[pred] + w(pred,t) bit-exact, hops += 1) and
    # no shorter relaxation through any in-arc (lat[t] <= lat[u] + w)
    f, t = top.normalized_endpoints()
    nl = f != t
    W = {}
    for a, b, w in zip(f[nl], t[nl], top.latency[nl]):
        W[(int(a), int(b))] = w
    import scipy.sparse as sp
    A = sp.coo_matrix((top.latency[nl], (f[nl], t[nl])), shape=(top.n, top.n)).tocsr()
    A = (A + A.T).tocsr()
    for s in att[::997]:
        r = eng.get_row(int(s))
        lat, hops, pred = r["lat"], r["hops"], r["pred"]
        for tt in range(0, top.n, 37):
            if tt == s:
                continue
            p = pred[tt]
            w = W[(max(p, tt), min(p, tt))]
            assert lat[tt] == lat[p] + w if p != s else lat[tt] == 0.0 + w
            assert hops[tt] == (hops[p] + 1 if p != s else 1)
        coo = A.tocoo()
        cand = np.where(coo.row == s, 0.0, lat[coo.row]) + coo.data
        assert np.all(lat[coo.col][coo.col != s] <= cand[coo.col != s])
    eng.close()


def test_dense_minplus_shipped_minus_one(E, oracle_mod):
    """K2 dense path on the shipped graph minus one edge (isComplete FALSE):
    0.005-quantised latencies -> many tie rows resolved by the exact kernel."""
    top = Topology.load_npz(os.path.join(GOLDEN, "shipped_topology.npz"))
    m1 = G.minus_one_edge(top, seed=3)
    st = _check_engine(E, oracle_mod, m1, np.arange(top.n))
    assert st["mode"] == 3 and st["launchesDense"] >= 1
    assert st["rowsExact"] > 0


@pytest.mark.parametrize("n,seed", [(700, 3), (1200, 5)])
def test_dense_minplus_random(E, oracle_mod, n, seed):
    top = G.dense(n, seed=seed, drop_edge=True)
    st = _check_engine(E, oracle_mod, top, np.arange(n), sources=np.arange(0, n, 9))
    assert st["mode"] == 3 and st["denseSweeps"] >= 2


def test_dense_forced_on_sparse_graph(E, oracle_mod):
    top = G.random_sparse(300, 6, seed=44, vloss=True)
    st = _check_engine(E, oracle_mod, top, np.arange(300), force=4)
    assert st["mode"] == 3


@pytest.mark.parametrize("case", ["tiefree", "directed", "vloss", "quantized", "power_law",
                                  "rgg_partial", "missing_loop"])
def test_batched_kernel(E, oracle_mod, case):
    """Batched multi-source kernel (forceMode 5, pe_batch.hip) vs the oracle."""
    if case == "tiefree":
        top, att, srcs = G.random_sparse(500, 5, seed=201), np.arange(500), None
    elif case == "directed":
        top, att, srcs = G.random_sparse(400, 4, seed=202, directed=True), np.arange(400), None
    elif case == "vloss":
        top, att, srcs = G.random_sparse(400, 4, seed=203, vloss=True), np.arange(0, 400, 3), None
    elif case == "quantized":
        top, att, srcs = G.random_sparse(400, 6, seed=204, quantum=1.0), np.arange(400), None
    elif case == "power_law":
        top = G.power_law(6000, m=3, seed=4)
        att = G.sample_attached(top.n, 1000, seed=2)
        srcs = att[::7]
    elif case == "rgg_partial":
        top = G.rgg(3000, seed=9)
        att = G.sample_attached(top.n, 700, seed=1)
        srcs = att[::3]
    else:
        src = np.array([0, 1, 2, 3, 0, 2, 3])
        dst = np.array([1, 2, 0, 0, 0, 2, 3])
        top = Topology(4, True, src, dst, np.array([1.0, 2.0, 3.0, 4.0, 0.5, 0.5, 0.5]),
                       np.zeros(7))
        att, srcs = np.arange(4), None
    st = _check_engine(E, oracle_mod, top, att, sources=srcs, force=5)
    assert st["mode"] == 1 and st["launchesSparse"] >= 1
    if case == "quantized":
        assert st["rowsExact"] > 0
        assert st["rowsTieEarly"] > 0      # early-stop emulation + k_tie_write


def _chain(n, seed, vloss=False):
    """Path graph 0-1-...-(n-1) with self-loops: one tree, depth up to n-1."""
    rng = np.random.default_rng(seed)
    src = np.concatenate([np.arange(n - 1), np.arange(n)])
    dst = np.concatenate([np.arange(1, n), np.arange(n)])
    m = src.shape[0]
    return Topology(n, False, src, dst, rng.uniform(1.0, 50.0, m), rng.uniform(0.0, 0.02, m),
                    rng.uniform(0.0, 0.01, n) if vloss else None)


@pytest.mark.parametrize("n,vloss", [(4400, False), (300, True), (1500, True)])
def test_batched_kernel_deep_trees(E, oracle_mod, n, vloss):
    """Deep predecessor trees in k_batch_rows: many pointer-jumping rounds,
    depth > LMAX (4096: Gauss-Seidel reliability sweeps) and, with vertex
    loss, the chain fold of fold_rel_batch beyond 64 hops."""
    top = _chain(n, seed=n, vloss=vloss)
    att = np.arange(n, dtype=np.int32)
    srcs = np.array([0, n - 1, n // 2, n // 3, 7], np.int32)
    st = _check_engine(E, oracle_mod, top, att, sources=srcs, force=5)
    assert st["mode"] == 1 and st["rowsExact"] == 0


def test_native_graphml_to_engine(E, oracle_mod):
    """§8 f4 end to end: shipped GraphML -> shd_graphml_parse -> shd_pe_create
    (complete graph: direct rows), and the same file minus one edge (Dijkstra
    rows), both bit-exact against the oracle."""
    path = os.path.join(os.path.dirname(__file__), "data", "topology.graphml.xml.xz")
    top = E.parse_graphml(path)
    att = np.arange(top.n, dtype=np.int32)
    og = oracle_mod.OracleGraph(top)
    eng = E.Engine(top, att)
    assert eng.is_complete
    eng.compute_all()
    for s in (0, 91, 182):
        r = eng.get_row(s)
        assert np.all(r["flags"] == E.F_DIRECT)
        for t in range(top.n):
            lat, rel = og.direct(s, t)
            assert r["lat"][t] == lat and r["rel"][t] == rel
    assert eng.stats()["mode"] == 2
    eng.close()
    keep = np.ones(top.m, bool)
    keep[np.flatnonzero(top.src != top.dst)[0]] = False
    cut = Topology(top.n, top.directed, top.src[keep], top.dst[keep], top.latency[keep],
                   top.loss[keep], top.vloss)
    st = _check_engine(E, oracle_mod, cut, att, sources=att[::5])
    assert st["mode"] != 2


def _ladder(k, seed, vloss=False, directed=False):
    """Two chains 0..k-1 and k..2k-1 with rungs i <-> k+i, all latencies 1:
    every vertex beyond the first rung has equal-distance predecessors, so
    every row is a tie row with ties at depth up to ~k (long chains for the
    blocked reliability fold)."""
    rng = np.random.default_rng(seed)
    a = np.arange(k - 1)
    src = np.concatenate([a, a + k, np.arange(k), np.arange(2 * k)])
    dst = np.concatenate([a + 1, a + 1 + k, np.arange(k) + k, np.arange(2 * k)])
    m = src.shape[0]
    return Topology(2 * k, directed, src, dst, np.ones(m), rng.uniform(0.0, 0.02, m),
                    rng.uniform(0.0, 0.01, 2 * k) if vloss else None)


@pytest.mark.parametrize("k,vloss,directed", [(150, True, False), (350, False, False),
                                              (120, True, True)])
def test_batched_tie_rows_early_stop(E, oracle_mod, k, vloss, directed):
    """Every row is a tie row: the batch kernel exports distances, parents and
    the tie threshold; k_exact_rows stops at the threshold and k_tie_write
    folds hops / reliability (vertex loss: blocked chain fold beyond 64
    hops).  2k > 254 rows overflow the tie slots: the rest take the full
    heap emulation, both must match the oracle."""
    top = _ladder(k, seed=k, vloss=vloss, directed=directed)
    att = np.arange(2 * k, dtype=np.int32)
    st = _check_engine(E, oracle_mod, top, att, force=5)
    assert st["mode"] == 1 and st["rowsExact"] > 0
    assert st["rowsTieEarly"] > 0
    if 2 * k > 254:
        assert st["rowsTieEarly"] < st["rowsExact"]


def test_batched_tie_rows_partial_targets(E, oracle_mod):
    """Quantised latencies with 1 of 5 vertices attached: ambiguous entries
    off every target's path are cleared by the relevance scan (fast-path
    parents kept), the rest run the early-stop emulation."""
    top = G.random_sparse(3000, 5, seed=77, quantum=1.0)
    att = np.arange(0, 3000, 5, dtype=np.int32)
    st = _check_engine(E, oracle_mod, top, att, force=5)
    assert st["mode"] == 1 and st["rowsTieEarly"] > 0


def test_topology_shim_concurrent_readers(E, oracle_mod):
    """8 host threads query the topology mirror at once (the reference's
    worker threads): cache hits take no lock, misses serialise.  Every value
    is the engine row entry of one of the two directions (whichever row was
    computed first -- the reference's cache keeps the first), the cache
    holds one entry per unordered pair, and packet counters add up."""
    import threading
    top = G.random_sparse(800, 5, seed=41, vloss=True)
    att = np.arange(0, 800, 3, dtype=np.int32)
    eng = E.Engine(top, att)
    shim = E.TopologyShim(eng)
    pos = {int(v): j for j, v in enumerate(att)}
    eng.compute_rows(att)
    rows = {int(s): eng.get_row(int(s)) for s in att}
    errors, incs = [], [0] * 8

    def worker(i):
        r = np.random.default_rng(500 + i)
        for _ in range(4000):
            s, d = (int(x) for x in r.choice(att, 2))
            if s == d:
                continue
            lat = shim.get_latency(s, d)
            ok = (lat == rows[s]["lat"][pos[d]] or lat == rows[d]["lat"][pos[s]])
            if not ok:
                errors.append((s, d, lat))
            if shim.increment(s, d) == 0:
                incs[i] += 1

    th = [threading.Thread(target=worker, args=(i,)) for i in range(8)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors[:5]
    total, seen = 0, 0
    for a in att:
        for b in att:
            c1, c2 = shim.cached(int(a), int(b)), shim.cached(int(b), int(a))
            assert a == b or not (c1 and c2)
            if c1:
                total += c1[3]
                seen += 1
    assert total == sum(incs)
    assert seen == shim.cache_size
    shim.close()
    eng.close()


@pytest.mark.parametrize("n", [650_000, 660_000, 800_000])
def test_large_graph_batched_kernel(E, oracle_mod, n):
    """k_batch_rows keeps its two pending bitmaps in LDS up to 655,104
    vertices (160 KB); past that they live in the slot's HBM scratch (the
    reference runs igraph Dijkstra at any size, topology.c:1765).  Both
    sides of the switch and an 800k-vertex graph: rows bit-exact against
    the oracle."""
    rng = np.random.default_rng(n)
    perm = rng.permutation(n)
    extra = rng.integers(0, n, size=(n, 2))
    src = np.concatenate([perm[:-1], extra[:, 0]])
    dst = np.concatenate([perm[1:], extra[:, 1]])
    key = np.minimum(src, dst).astype(np.int64) * n + np.maximum(src, dst)
    _, first = np.unique(key, return_index=True)
    keep = np.zeros(src.shape[0], bool)
    keep[first] = True
    keep &= src != dst
    src, dst = src[keep], dst[keep]
    top = Topology(n, False, src, dst, rng.uniform(1.0, 50.0, src.shape[0]),
                   rng.uniform(0.0, 0.02, src.shape[0]))
    att = np.array([0, n // 3, n // 2, n - 1], np.int32)
    st = _check_engine(E, oracle_mod, top, att)
    assert st["mode"] == 1 and st["batched"] == 1


def test_tune_picks_a_variant_and_keeps_parity(E, oracle_mod):
    """shd_pe_tune times both k_batch_rows variants (8 / 4 waves per SIMD)
    on the engine's rows and keeps the faster; the table it leaves and every
    later compute stay bit-exact."""
    top = G.power_law(30_000, 3, seed=5)
    att = np.arange(0, top.n, 7, dtype=np.int32)
    eng = E.Engine(top, att, force_mode=5)
    eng.tune()
    st = eng.stats()
    assert st["batched"] == 1 and st["batchWaves"] in (4, 6, 8) and st["rowsComputed"] == 0
    assert st["batchPostWaves"] in (4, 6, 8)
    og = oracle_mod.OracleGraph(top)
    pos = np.arange(0, eng.T, 97)
    exp = og.rows(eng.attached[pos], eng.attached, threads=8)
    for rnd in range(2):               # the tuned table, then a fresh compute
        for i, p in enumerate(pos):
            got = {k: (v[0] if v is not None else None) for k, v in eng.get_rows(int(p), 1).items()}
            _assert_rows_equal(got, {k: v[i] for k, v in exp.items()}, f"round {rnd} row {p}")
        eng.compute_all()
    eng.close()


@pytest.mark.parametrize("wpe", [4, 6, 8])
def test_tune_never_picks_a_failing_variant(E, oracle_mod, monkeypatch, wpe):
    """A variant whose batches fail their checks (SHDPE_TUNE_FAIL_WPE: its
    relax flags every batch, as the miscompiled post kernel of round 6's
    r05au record did) looks faster to the tune -- its skipped phases are not
    in the batch-kernel time -- but sends every row to the exact path: the
    tune excludes it for both kernels, and the table it leaves is computed
    on the fast path, bit-exact."""
    monkeypatch.setenv("SHDPE_TUNE_FAIL_WPE", str(wpe))
    top = G.power_law(8000, m=3, seed=14)
    att = G.sample_attached(top.n, 1200, seed=3)
    eng = E.Engine(top, att, force_mode=5, debug_flags=E.DEBUG_ENV)
    eng.tune()
    st = eng.stats()
    assert st["batched"] == 1 and st["batchWaves"] != wpe and st["batchPostWaves"] != wpe, st
    eng.compute_all()
    st = eng.stats()
    assert st["rowsExact"] == 0, st
    og = oracle_mod.OracleGraph(top)
    pos = np.arange(0, eng.T, 37)
    exp = og.rows(eng.attached[pos], eng.attached, threads=8)
    for i, p in enumerate(pos):
        got = {k: (v[0] if v is not None else None) for k, v in eng.get_rows(int(p), 1).items()}
        _assert_rows_equal(got, {k: v[i] for k, v in exp.items()}, f"row {p}")
    eng.close()


@pytest.mark.parametrize("wpe", [4, 6, 8])
@pytest.mark.parametrize("case", ["power_law", "quantized"])
def test_batched_kernel_each_variant(E, oracle_mod, monkeypatch, wpe, case):
    """Every k_batch_rows variant the tune may pick (4 / 6 / 8 waves per
    SIMD; 6 = two 768-thread workgroups per CU) forced through
    SHDPE_BATCH_WPE, bit-exact with the oracle, tie rows included."""
    monkeypatch.setenv("SHDPE_BATCH_WPE", str(wpe))
    if case == "power_law":
        top = G.power_law(8000, m=3, seed=14)
        att = G.sample_attached(top.n, 1200, seed=3)
        srcs = att[::5]
    else:
        top, att, srcs = G.random_sparse(600, 6, seed=214, quantum=1.0), np.arange(600), None
    st = _check_engine(E, oracle_mod, top, att, sources=srcs, force=5, debug_flags=E.DEBUG_ENV)
    assert st["batched"] == 1 and st["batchWaves"] == wpe
    if case == "quantized":
        assert st["rowsExact"] > 0


@pytest.mark.parametrize("lb", [4, 8, 16, 32])
@pytest.mark.parametrize("wpe", [4, 8])
@pytest.mark.parametrize("case", ["power_law", "quantized"])
def test_batched_kernel_each_lb(E, oracle_mod, monkeypatch, lb, wpe, case):
    """Every batch width the engine may pick by shard size (LB 16 / 8 / 4
    sources per batch: 8-GPU shards of C4 take LB 4), forced through
    SHDPE_BATCH_LB at both register budgets, bit-exact with the oracle, tie
    rows and a ragged last batch included."""
    monkeypatch.setenv("SHDPE_BATCH_LB", str(lb))
    monkeypatch.setenv("SHDPE_BATCH_WPE", str(wpe))
    if case == "power_law":
        top = G.power_law(8000, m=3, seed=15)
        att = G.sample_attached(top.n, 1203, seed=4)
        srcs = att[::3]
    else:
        top, att, srcs = G.random_sparse(600, 6, seed=215, quantum=1.0), np.arange(599), None
    st = _check_engine(E, oracle_mod, top, att, sources=srcs, force=5, debug_flags=E.DEBUG_ENV)
    assert st["batched"] == 1 and st["batchLanes"] == lb and st["batchWaves"] == wpe
    if case == "quantized":
        assert st["rowsExact"] > 0
    else:
        # tie-free: a batch reaches the exact kernel only if its relaxation
        # failed (a group barrier timed out, or near vertices were lost and
        # the post kernel's Bellman check fired) -- the phase-alternating
        # publication buffers keep that from happening
        assert st["rowsExact"] == 0


@pytest.mark.parametrize("lb", [8, 16])
@pytest.mark.parametrize("wpe", [4, 6, 8])
@pytest.mark.parametrize("case", ["power_law", "quantized"])
def test_cooperative_relax_each_variant(E, oracle_mod, monkeypatch, lb, wpe, case):
    """The cooperative relax (two workgroups of one XCD share a batch: dist
    array at agent scope, near bits published per listing round, group
    barriers) forced at every batch width and variant it exists for: every
    row bit-exact with the oracle, no batch failed its Bellman check (a lost
    update would send it to the exact kernel), no launch aborted."""
    monkeypatch.setenv("SHDPE_BATCH_LB", str(lb))
    monkeypatch.setenv("SHDPE_BATCH_COOP", "2")
    monkeypatch.setenv("SHDPE_BATCH_COOP_WPE", str(wpe))
    if case == "power_law":
        top = G.power_law(8000, m=3, seed=15)
        att = G.sample_attached(top.n, 1203, seed=4)
        srcs = att[::3]
    else:
        top, att, srcs = G.random_sparse(600, 6, seed=215, quantum=1.0), np.arange(599), None
    st = _check_engine(E, oracle_mod, top, att, sources=srcs, force=5, debug_flags=E.DEBUG_ENV)
    assert st["batched"] == 1 and st["batchLanes"] == lb and st["batchCoop"] == 2, st
    assert st["relaxCoopAborts"] == 0, st
    if case == "quantized":
        assert st["rowsExact"] > 0, st
    else:
        assert st["rowsExact"] == 0, st


def test_cooperative_relax_abort_recomputes(E, oracle_mod, monkeypatch):
    """A cooperative launch whose barrier waits give up at once
    (SHDPE_COOP_SPIN=0: the first wait that is not already satisfied aborts
    the launch) is recomputed by the plain relax: the aborts are counted and
    every row is still bit-exact -- never a wrong or missing row."""
    monkeypatch.setenv("SHDPE_BATCH_LB", "8")
    monkeypatch.setenv("SHDPE_BATCH_COOP", "2")
    monkeypatch.setenv("SHDPE_COOP_SPIN", "0")
    top = G.power_law(8000, m=3, seed=15)
    att = G.sample_attached(top.n, 1203, seed=4)
    st = _check_engine(E, oracle_mod, top, att, sources=att[::3], force=5, debug_flags=E.DEBUG_ENV)
    assert st["batchCoop"] == 2 and st["relaxCoopAborts"] >= 1 and st["rowsExact"] == 0, st


@pytest.mark.parametrize("mode", ["1", "2"])
@pytest.mark.parametrize("case", ["batched", "sparse"])
def test_tie_slot_cross_check_repairs(E, oracle_mod, monkeypatch, case, mode):
    """Early-stop tie rows: the exact kernel checks every vertex it popped
    against the exported distance of the same row (a slot holding another
    source's or a stale distance array -- the round-4 r04t symptom, latencies
    below the true distance -- fails it), and k_tie_write writes no row from
    an array whose own source is not at distance 0 (the latency floor).
    SHDPE_TIE_CORRUPT=1 halves one slot's exported distances after the
    relevance scan, =2 shifts them all by 1 ms: the row must be caught
    (rowsTieRepaired), recomputed by the full emulation, and every row stays
    bit-exact with the oracle."""
    monkeypatch.setenv("SHDPE_TIE_CORRUPT", mode)
    if case == "batched":
        top, att, force = G.random_sparse(600, 6, seed=216, quantum=1.0), np.arange(599), 5
    else:
        top, att, force = G.rgg(2000, seed=9, quantum=0.05), None, 1
        att = np.arange(top.n, dtype=np.int32)
    st = _check_engine(E, oracle_mod, top, att, force=force, debug_flags=E.DEBUG_ENV)
    assert st["rowsTieEarly"] > 0 and st["rowsTieRepaired"] >= 1, st


def test_deferred_tie_export_violation_takes_full_emulation(E, oracle_mod, monkeypatch):
    """The batched path's deferred tie export (k_tie_export, after the post
    kernel) re-checks every in-arc of every vertex of a tie row's distance
    array; a Bellman violation there must send that row to the full igraph
    emulation instead of the early-stop one.  SHDPE_TIE_CORRUPT=3 makes the
    export treat its first slot as violated: one early-stop row fewer, the
    same rows to the exact path, every row still bit-exact with the oracle."""
    top, att = G.random_sparse(600, 6, seed=216, quantum=1.0), np.arange(599)
    base = _check_engine(E, oracle_mod, top, att, force=5, debug_flags=E.DEBUG_ENV)
    monkeypatch.setenv("SHDPE_TIE_CORRUPT", "3")
    st = _check_engine(E, oracle_mod, top, att, force=5, debug_flags=E.DEBUG_ENV)
    assert base["rowsTieEarly"] >= 1, base
    assert st["rowsExact"] == base["rowsExact"], (base, st)
    assert st["rowsTieEarly"] == base["rowsTieEarly"] - 1, (base, st)


def test_tune_with_fewer_scratch_slots_than_grid(E, oracle_mod, monkeypatch):
    """A scratch budget below the resident grid (huge graphs, or a small
    SHDPE_BATCH_SCRATCH_GB): shd_pe_tune must time its variants -- and keep
    one -- with grids no larger than the slots allocated (a workgroup indexes
    its slot by blockIdx); rows stay bit-exact."""
    monkeypatch.setenv("SHDPE_BATCH_SCRATCH_GB", "0.3")     # ~25 slots of a 30k-vertex graph
    top = G.power_law(30_000, 3, seed=6)
    att = np.arange(0, top.n, 11, dtype=np.int32)
    eng = E.Engine(top, att, force_mode=5, debug_flags=E.DEBUG_ENV)
    eng.tune()
    eng.compute_all()
    og = oracle_mod.OracleGraph(top)
    pos = np.arange(0, eng.T, 61)
    exp = og.rows(eng.attached[pos], eng.attached, threads=8)
    for i, p in enumerate(pos):
        got = {k: (v[0] if v is not None else None) for k, v in eng.get_rows(int(p), 1).items()}
        _assert_rows_equal(got, {k: v[i] for k, v in exp.items()}, f"row {p}")
    eng.close()


def _oracle_path(top, og, s, t, att):
    """igraph's path s -> t from the oracle's raw Dijkstra (parent edge ids)."""
    _, par, _ = og.raw(int(s), att)
    path, v = [int(t)], int(t)
    while v != s:
        e = int(par[v]) - 1
        assert e >= 0, "unreached"
        a, b = int(top.src[e]), int(top.dst[e])
        v = a if (top.directed or b == v) else b
        path.append(v)
    return path[::-1]


@pytest.mark.parametrize("case", ["tiefree", "quantized", "directed", "batched"])
def test_get_path_matches_igraph(E, oracle_mod, case):
    """shd_pe_get_path: the vertex sequence topology.c prints hop by hop
    (:1449, :1502-1503) -- igraph's path, ties decided by its heap."""
    if case == "directed":
        top = G.random_sparse(700, 5, seed=31, directed=True)
    elif case == "quantized":
        top = G.random_sparse(800, 5, seed=32, quantum=0.5)
    elif case == "batched":
        top = G.power_law(3000, 3, seed=33, quantum=0.25)
    else:
        top = G.random_sparse(800, 5, seed=34)
    att = np.arange(0, top.n, 3, dtype=np.int32)
    eng = E.Engine(top, att, force_mode=5 if case == "batched" else 0)
    og = oracle_mod.OracleGraph(top)
    rng = np.random.default_rng(5)
    checked = 0
    for s in rng.choice(att, 4, replace=False):
        for t in rng.choice(att, 6, replace=False):
            if s == t:
                assert eng.get_path(int(s), int(t)) == [int(s)]
                continue
            dist, _, _ = og.raw(int(s), att)
            if dist[t] < 0:
                with pytest.raises(E.EngineError):
                    eng.get_path(int(s), int(t))
                continue
            got = eng.get_path(int(s), int(t))
            assert got == _oracle_path(top, og, s, t, att), (case, s, t)
            checked += 1
        eng.compute_all()                 # invalidates the cached parent array
    assert checked >= 10
    s0, t0 = int(att[0]), int(att[-1])
    with pytest.raises(E.EngineError):
        eng.get_path(s0, t0, cap=1)
    with pytest.raises(E.EngineError):
        eng.get_path(s0, 1)               # vertex 1 is not attached
    eng.close()


@pytest.mark.parametrize("force_mode", [0, 5])
def test_get_path_unreachable_is_eunreachable(E, force_mode):
    """Two disjoint components: a target in the other one has no parent chain.
    shd_pe_get_path must say SHD_PE_EUNREACHABLE (from the row's flags), never
    walk the stale scratch parents left there by an earlier row."""
    a, b = G.random_sparse(300, 4, seed=41), G.random_sparse(200, 4, seed=42)
    top = Topology(n=500, directed=False, src=np.concatenate([a.src, b.src + 300]),
                   dst=np.concatenate([a.dst, b.dst + 300]),
                   latency=np.concatenate([a.latency, b.latency]),
                   loss=np.concatenate([a.loss, b.loss]))
    att = np.arange(0, 500, 5, dtype=np.int32)
    eng = E.Engine(top, att, force_mode=force_mode)
    eng.compute_all()
    for s, t in ((0, 305), (310, 5), (5, 400), (450, 10)):
        assert eng.get_path(10, 20)[0] == 10           # leaves a full parent array behind
        with pytest.raises(E.EngineError) as ei:
            eng.get_path(s, t)
        assert ei.value.code == E.EUNREACHABLE, (s, t, ei.value)
    assert eng.get_path(305, 400)[-1] == 400
    eng.close()


def _twin_tie_graph(z_attached, seed=11):
    """A tie-free random graph plus twins a, b (both hanging off hub h with
    the same latency) and z adjacent to exactly a and b with equal latency:
    for every other source z has two equal-minimum tight predecessors (the
    heap decides its parent), and z is a leaf."""
    base = G.random_sparse(600, 5, seed=seed)
    n0 = base.n
    a, b, z, h = n0, n0 + 1, n0 + 2, 0
    src = np.concatenate([base.src, [h, h, a, b, a, b, z]])
    dst = np.concatenate([base.dst, [a, b, z, z, a, b, z]])
    lat = np.concatenate([base.latency, [7.25, 7.25, 3.5, 3.5, 1.0, 1.0, 1.0]])
    loss = np.concatenate([base.loss, [0.01, 0.01, 0.0, 0.0, 0.0, 0.0, 0.0]])
    top = Topology(n0 + 3, False, src, dst, lat, loss, None)
    att = np.arange(0, n0, 3, dtype=np.int32)
    if z_attached:
        att = np.concatenate([att, [z]]).astype(np.int32)
    return top, att


@pytest.mark.parametrize("z_attached", [False, True])
def test_batched_tie_relevance(E, oracle_mod, z_attached):
    """k_batch_rows sends a row to the exact path only when an ambiguous
    entry lies on a target's path: with z (ambiguous in every row but a's,
    b's and z's own) off every target path all rows stay on the fast path;
    with z a target every row is a tie row.  Bit-exact either way."""
    top, att = _twin_tie_graph(z_attached)
    st = _check_engine(E, oracle_mod, top, att, force=5)
    assert st["batched"] == 1
    if z_attached:
        assert st["rowsExact"] >= len(att) - 1
    else:
        assert st["rowsExact"] == 0
