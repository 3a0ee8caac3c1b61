"""Batched device helpers (pe_aux.hip) against the
oracle's one-query restatements of topology.c:

  shd_pe_self_paths          _topology_computeShortestPathToSelf  :1545-1653
  shd_pe_direct_paths        _topology_lookupDirectPath           :1877-1927
  shd_pe_adjacent_pairs      _topology_verticesAreAdjacent        :1248-1264
  shd_pe_is_complete_device  _topology_isComplete                 :450-552

Bit-exact comparisons (lat, rel are f64 gathers / one product chain)."""
import os

import numpy as np
import pytest

from shdpe import generators as G
from shdpe.graph import Topology

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def E():
    from shdpe import engine
    return engine


def _drop_some_loops(top, seed):
    """Remove the self-loop of every 3rd vertex (missing (s,s) edges)."""
    rng = np.random.default_rng(seed)
    loops = np.flatnonzero(top.src == top.dst)
    drop = loops[rng.random(loops.shape[0]) < 0.33]
    keep = np.ones(top.m, bool)
    keep[drop] = False
    return Topology(n=top.n, directed=top.directed, src=top.src[keep], dst=top.dst[keep],
                    latency=top.latency[keep], loss=top.loss[keep], vloss=top.vloss,
                    name=top.name + "_someloops")


def _graphs():
    yield "quantised_ties", G.random_sparse(700, 8, seed=3, quantum=10.0)
    yield "directed_vloss", G.random_sparse(500, 6, seed=4, directed=True, vloss=True)
    yield "missing_loops", _drop_some_loops(G.random_sparse(600, 5, seed=5, quantum=5.0), 1)
    yield "power_law", G.power_law(5000, m=3, seed=7, quantum=0.5)
    yield "multigraph", G.with_parallel_edges(G.random_sparse(500, 6, seed=12, vloss=True, quantum=5.0), 0.3, seed=5)
    yield "multigraph_directed", G.with_parallel_edges(G.random_sparse(400, 6, seed=13, directed=True), 0.3, seed=6)
    yield "parallel_loops", G.with_parallel_loops(G.random_sparse(400, 6, seed=14, quantum=5.0), 0.6, seed=8)
    yield "parallel_loops_directed", G.with_parallel_loops(G.random_sparse(300, 6, seed=15, directed=True), 0.6, seed=9)
    yield "newest_slower", G.with_slower_newest_edges(G.random_sparse(400, 6, seed=16, quantum=5.0), 0.4, seed=12)
    yield "newest_slower_directed", G.with_slower_newest_edges(G.random_sparse(300, 6, seed=17, directed=True), 0.4, seed=13)


@pytest.mark.parametrize("name,top", list(_graphs()), ids=[n for n, _ in _graphs()])
def test_self_paths_match_oracle(E, oracle_mod, name, top):
    eng = E.Engine(top, np.arange(min(top.n, 64), dtype=np.int32))
    og = oracle_mod.OracleGraph(top)
    verts = np.concatenate([np.arange(top.n), [-1, top.n]]).astype(np.int32)
    lat, rel, flags = eng.self_paths(verts)
    for i, v in enumerate(verts[:-2]):
        exp = og.self_path(int(v))
        assert exp is not None
        assert flags[i] == 0, (name, v)
        assert lat[i] == exp[0] and rel[i] == exp[1], (name, v, lat[i], rel[i], exp)
        assert (lat[i], rel[i]) == eng.self_path(int(v))
    assert flags[-1] == E.F_INVALID and flags[-2] == E.F_INVALID
    eng.close()


@pytest.mark.parametrize("name,top", list(_graphs()), ids=[n for n, _ in _graphs()])
def test_direct_paths_and_adjacency_match_oracle(E, oracle_mod, name, top):
    eng = E.Engine(top, np.arange(min(top.n, 64), dtype=np.int32))
    og = oracle_mod.OracleGraph(top)
    rng = np.random.default_rng(11)
    k = 20000
    src = rng.integers(0, top.n, k).astype(np.int32)
    dst = rng.integers(0, top.n, k).astype(np.int32)
    # every edge (both directions), every loop position, and invalid ids
    src = np.concatenate([src, top.src, top.dst, np.arange(top.n), [-1, 0, top.n]]).astype(np.int32)
    dst = np.concatenate([dst, top.dst, top.src, np.arange(top.n), [0, -1, 0]]).astype(np.int32)
    lat, rel, flags = eng.direct_paths(src, dst)
    adj = eng.adjacent_pairs(src, dst)
    for i in range(src.shape[0]):
        s, t = int(src[i]), int(dst[i])
        if s < 0 or t < 0 or s >= top.n or t >= top.n:
            assert flags[i] == E.F_INVALID and adj[i] == 0
            continue
        exp = og.direct(s, t)
        if exp is None:
            assert flags[i] == E.F_NOEDGE and adj[i] == 0, (name, s, t)
        else:
            assert flags[i] == E.F_DIRECT and adj[i] == 1, (name, s, t)
            assert lat[i] == exp[0] and rel[i] == exp[1], (name, s, t)
        assert bool(adj[i]) == (og.get_eid(s, t) != -1)
    eng.close()


def test_is_complete_device(E, oracle_mod):
    top = Topology.load_npz(os.path.join(ROOT, "tests", "golden", "shipped_topology.npz"),
                            name="shipped")
    for t in (top, G.minus_one_edge(top, seed=3), G.dense(300, seed=2),
              G.dense(300, seed=2, drop_edge=True), G.random_sparse(200, 4, seed=1),
              G.with_parallel_edges(G.dense(100, seed=2, drop_edge=True), 0.2, seed=3),
              G.with_parallel_edges(G.random_sparse(200, 4, seed=1), 0.5, seed=4)):
        eng = E.Engine(t, np.arange(min(t.n, 32), dtype=np.int32))
        og = oracle_mod.OracleGraph(t)
        assert eng.is_complete_device() == og.is_complete() == bool(eng.stats()["isComplete"])
        eng.close()


def test_batched_pairs_chunking(E, oracle_mod):
    """More pairs than one staging chunk would hold at small sizes: a large
    call on the shipped complete graph equals the per-pair helper."""
    top = Topology.load_npz(os.path.join(ROOT, "tests", "golden", "shipped_topology.npz"),
                            name="shipped")
    eng = E.Engine(top, np.arange(top.n, dtype=np.int32))
    s, t = np.meshgrid(np.arange(top.n, dtype=np.int32), np.arange(top.n, dtype=np.int32))
    s, t = s.ravel(), t.ravel()
    lat, rel, flags = eng.direct_paths(s, t)
    assert np.all(flags == E.F_DIRECT)
    for i in range(0, s.shape[0], 97):
        assert (lat[i], rel[i]) == eng.direct_path(int(s[i]), int(t[i]))
    eng.close()


def _fill_cases():
    yield "missing_loops", _drop_some_loops(G.random_sparse(600, 5, seed=21, quantum=5.0), 2), 0
    yield "directed", G.random_sparse(500, 3, seed=22, directed=True, vloss=True), 0
    yield "batched", G.power_law(20_000, m=3, seed=23), 5
    yield "complete", G.dense(80, seed=24), 0


@pytest.mark.parametrize("name,top,force", list(_fill_cases()), ids=[n for n, _, _ in _fill_cases()])
def test_fill_rowstore_equals_store_rows(E, name, top, force):
    """shd_pe_fill_rowstore (device-packed triangular image + one DMA) leaves
    the row store exactly as shd_rowstore_store_rows over every engine row in
    position order: same entries in the same direction, size, minimum
    latency, per-row results -- unreachable targets, missing self-loops
    (F_NOEDGE), directed reverse entries and complete graphs (nothing
    non-direct stored) included."""
    att = np.arange(top.n, dtype=np.int32) if top.n <= 1000 else G.sample_attached(top.n, 900, seed=4)
    eng = E.Engine(top, att, force_mode=force)
    eng.compute_all()
    rows = eng.get_rows(0, eng.T)
    ref = E.RowStore(top.n, eng.attached)
    rr = ref.store_rows(eng.attached, rows["lat"], rows["rel"], rows["flags"], is_complete=eng.is_complete)
    st = E.RowStore(top.n, eng.attached)
    res, ms = eng.fill_rowstore(st)
    assert np.array_equal(res, np.asarray(rr, np.int32))
    assert st.size() == ref.size() and st.min_latency() == ref.min_latency()
    assert sorted(st.items()) == sorted(ref.items())
    if name == "complete":
        assert st.size() == 0                       # (still empty: a second fill is legal)
    else:
        with pytest.raises(E.EngineError):
            eng.fill_rowstore(st)                   # the store is no longer empty
    st.close()
    ref.close()
    eng.close()


def test_fill_rowstore_sharded_engine(E):
    """A multi-shard engine (logical shards on the test GPU) refuses the
    one-call fill with SHD_PE_ENOTOWNED until its rows are gathered (its
    host image is released on that path), then fills exactly as a
    one-shard engine does."""
    top = G.power_law(6_000, m=3, seed=25)
    att = G.sample_attached(top.n, 700, seed=4)
    one = E.Engine(top, att, force_mode=5)
    ref = E.RowStore(top.n, one.attached)
    rr, _ = one.fill_rowstore(ref)
    eng = E.Engine(top, att, force_mode=5, devices=[0, 0])
    st = E.RowStore(top.n, eng.attached)
    for _ in range(2):                              # (a repeat must not leak or crash)
        with pytest.raises(E.EngineError) as ei:
            eng.fill_rowstore(st)
        assert ei.value.code == E.ENOTOWNED
    assert st.size() == 0
    eng.gather()
    res, _ = eng.fill_rowstore(st)
    assert np.array_equal(res, rr)
    assert st.size() == ref.size() and st.min_latency() == ref.min_latency()
    assert sorted(st.items()) == sorted(ref.items())
    for x in (st, ref, eng, one):
        x.close()
