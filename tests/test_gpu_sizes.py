"""GPU parity at the BASELINE.json configuration sizes, through the C-ABI.

Semantics under test: topology.c:1655-1875 (Dijkstra rows: igraph 0.7.1
Dijkstra + _topology_computePathProperties fold) and :1877-1927 (direct rows
of complete graphs).  Bar: lat / rel bit-exact, hops / pred identical, failure
and zero-latency flags identical (stricter than north_star's 1e-12 relative).

Coverage per config (the oracle runs on 16 host threads, pipelined block by
block with the comparison):
  C2   the whole 10,000 x 10,000 table, and the whole C2q (tie) table
  C4   the whole 16,384 x 16,384 table (north_star target)
  C4q  every tie row + 256 random rows
  C5   2,048 random rows; every row of the table checked for failures,
       positivity and hop counts
  C5q  every tie row of the full table + 256 random rows
  C3a  the whole 20,000 x 20,000 direct table against the edge list
  C3b  256 rows bit-exact; predecessor consistency (lat[t] = lat[p] + w(p,t)
       bit-exact, hops[t] = hops[p] + 1) on EVERY row; the Bellman condition
       on every 100th row
  dense quantised (n = 3,000, 0.005 and 1 ms): every tie row + 256 rows
       bit-exact, Bellman on every row
The file sorts after test_gpu_parity.py / test_gpu_shards.py so a -x failure
in the quick cases stops the run before these.
"""
import os
import queue
import threading

import numpy as np
import pytest

from shdpe import generators as G

pytestmark = pytest.mark.gpu

REL_TOL = 1e-12
THREADS = min(16, os.cpu_count() or 1)
FLAG_SEM = 0x07          # unreachable | no edge | zero latency (F_EXACT / F_DIRECT are engine-side)


@pytest.fixture(scope="module")
def E():
    from shdpe import engine
    engine.load_library()
    return engine


def assert_block_equal(got, exp, ctx):
    """Rows of the engine vs the oracle, all fields, bit-exact."""
    assert np.array_equal(got["flags"] & FLAG_SEM, exp["flags"] & FLAG_SEM), f"{ctx} flags"
    ok = (exp["flags"] & 0x03) == 0
    for k in ("lat", "rel"):
        g, e = got[k][ok], exp[k][ok]
        bad = np.flatnonzero(g.view(np.int64) != e.view(np.int64))
        assert bad.size == 0, f"{ctx} {k}: {bad.size} entries differ, first {bad[:4]} got {g[bad[:3]]} exp {e[bad[:3]]}"
        assert np.allclose(g, e, rtol=REL_TOL, atol=0)
    for k in ("hops", "pred"):
        bad = np.flatnonzero(got[k][ok] != exp[k][ok])
        assert bad.size == 0, f"{ctx} {k}: {bad.size} entries differ, first {bad[:4]}"


def oracle_blocks(oracle_mod, top, sources, targets, block):
    """Yield (i0, rows) for consecutive blocks of `sources`, the oracle
    computing block b+1 on THREADS host threads (ctypes releases the GIL)
    while the caller compares block b."""
    og = oracle_mod.OracleGraph(top)
    q = queue.Queue(maxsize=1)
    err = []

    def producer():
        try:
            for i0 in range(0, sources.shape[0], block):
                q.put((i0, og.rows(sources[i0:i0 + block], targets, threads=THREADS)))
        except Exception as ex:       # noqa: BLE001 - re-raised in the consumer
            err.append(ex)
        q.put(None)

    th = threading.Thread(target=producer, daemon=True)
    th.start()
    while True:
        item = q.get()
        if item is None:
            break
        yield item
    th.join()
    if err:
        raise err[0]


def compare_positions(eng, oracle_mod, top, positions, ctx, block=512):
    """Engine rows at table positions `positions` vs the oracle."""
    positions = np.asarray(positions)
    srcs = eng.attached[positions]
    n = 0
    for i0, exp in oracle_blocks(oracle_mod, top, srcs, eng.attached, block):
        pos = positions[i0:i0 + block]
        if np.all(np.diff(pos) == 1):
            got = eng.get_rows(int(pos[0]), pos.shape[0])
        else:
            rows = [eng.get_rows(int(p), 1) for p in pos]
            got = {k: np.concatenate([r[k] for r in rows]) for k in rows[0]}
        assert_block_equal(got, exp, f"{ctx} rows {i0}..{i0 + pos.shape[0] - 1}")
        n += pos.shape[0]
    return n


def tie_positions(eng, E):
    """Table positions of the rows resolved by the exact path (F_EXACT)."""
    out = []
    for start in range(0, eng.T, 1024):
        blk = eng.get_rows(start, min(1024, eng.T - start))
        out += list(start + np.flatnonzero((blk["flags"] & E.F_EXACT).any(axis=1)))
    return np.array(out, np.int64)


def assert_fast_path(st, ctx, ties=False):
    """The rows came out of the fast kernels, not the safety nets: no tie row
    failed the exact kernel's slot cross-check (rowsTieRepaired), and no row
    went to the full igraph-heap emulation -- a tie-free table has no exact
    rows at all, a sparse tie table only early-stop tie rows (every row that
    fails the batch kernels' Bellman check goes to the full emulation, so a
    relax regression shows up here instead of only as a slower bench)."""
    assert st["rowsTieRepaired"] == 0, f"{ctx}: {st}"
    if not ties:
        assert st["rowsExact"] == 0, f"{ctx}: rows left the fast path: {st}"
    else:
        assert st["rowsExact"] == st["rowsTieEarly"], f"{ctx}: full-emulation rows: {st}"


def whole_table_properties(eng, ctx):
    """Every row: no failures (connected, self-loops), latency > 0,
    reliability in (0, 1], hops >= 1, pred a vertex id off the diagonal
    (the 1-vertex path [s] has no predecessor: pred -1, as the oracle)."""
    for start in range(0, eng.T, 1024):
        cnt = min(1024, eng.T - start)
        blk = eng.get_rows(start, cnt)
        assert not np.any(blk["flags"] & 0x03), f"{ctx} failed entries in rows {start}.."
        assert np.all(blk["lat"] > 0) and np.all((blk["rel"] > 0) & (blk["rel"] <= 1)), ctx
        assert np.all(blk["hops"] >= 1), ctx
        diag = np.zeros(blk["pred"].shape, bool)
        diag[np.arange(cnt), start + np.arange(cnt)] = True
        assert np.all(blk["pred"][~diag] >= 0), ctx
        assert np.all(blk["pred"][diag] == -1), ctx


# ---------------------------------------------------------------------------
# sparse configs
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("name", ["c2", "c2q"])
def test_c2_whole_table(E, oracle_mod, name):
    """C2 (RGG 10k, configs[1]) and its 0.005-quantised tie variant: every
    row of the table bit-exact against the oracle."""
    top, att = G.make_config(name)
    eng = E.Engine(top, att)
    eng.compute_all()
    st = eng.stats()
    assert st["rowsComputed"] == att.shape[0] and st["mode"] == 1
    if name == "c2q":
        assert st["rowsExact"] >= 1
    assert_fast_path(st, name, ties=name == "c2q")
    assert compare_positions(eng, oracle_mod, top, np.arange(eng.T), name, block=1000) == eng.T
    eng.close()


def test_c4_whole_table(E, oracle_mod):
    """C4 (BA n=100k, 16,384 attached; north_star target, k_batch_rows):
    all 16,384 x 16,384 entries bit-exact against the oracle."""
    top, att = G.make_config("c4")
    eng = E.Engine(top, att)
    eng.compute_all()
    st = eng.stats()
    assert st["rowsComputed"] == att.shape[0] and st["mode"] == 1 and st["batched"] == 1
    assert_fast_path(st, "c4")
    assert compare_positions(eng, oracle_mod, top, np.arange(eng.T), "c4", block=1024) == eng.T
    eng.close()


def test_c4q_tie_rows(E, oracle_mod):
    """C4 with latencies rounded to 0.005 ms: the whole table on the GPU;
    every tie row (F_EXACT: early-stop emulation + k_tie_write) and 256
    random rows bit-exact against the oracle's igraph-heap order."""
    top, att = G.make_config("c4q")
    eng = E.Engine(top, att)
    eng.compute_all()
    st = eng.stats()
    ties = tie_positions(eng, E)
    assert st["rowsExact"] > 0 and st["rowsTieEarly"] > 0
    assert 0 < ties.shape[0] <= st["rowsExact"]
    assert_fast_path(st, "c4q", ties=True)
    rng = np.random.default_rng(3)
    pos = np.unique(np.concatenate([ties, rng.choice(eng.T, 256, replace=False)]))
    compare_positions(eng, oracle_mod, top, pos, "c4q", block=256)
    eng.close()


def test_c5_sampled_rows(E, oracle_mod):
    """C5 (BA n=250k, 65,536 attached; 107 GB table on one GPU): 2,048 random
    rows bit-exact, every row checked for failures / positivity / hops."""
    top, att = G.make_config("c5")
    eng = E.Engine(top, att)
    eng.compute_all()
    st = eng.stats()
    assert st["rowsComputed"] == att.shape[0] and st["batched"] == 1
    assert_fast_path(st, "c5")
    rng = np.random.default_rng(11)
    pos = np.sort(rng.choice(eng.T, 2048, replace=False))
    compare_positions(eng, oracle_mod, top, pos, "c5", block=256)
    whole_table_properties(eng, "c5")
    eng.close()


def test_c5q_tie_rows(E, oracle_mod):
    """C5 with latencies rounded to 0.005 ms: the whole table on the GPU,
    every tie row and 256 random rows bit-exact."""
    top, att = G.make_config("c5q")
    eng = E.Engine(top, att)
    eng.compute_all()
    st = eng.stats()
    ties = tie_positions(eng, E)
    assert st["rowsExact"] > 0 and ties.shape[0] > 0
    assert_fast_path(st, "c5q", ties=True)
    rng = np.random.default_rng(5)
    pos = np.unique(np.concatenate([ties, rng.choice(eng.T, 256, replace=False)]))
    compare_positions(eng, oracle_mod, top, pos, "c5q", block=128)
    eng.close()


# ---------------------------------------------------------------------------
# dense configs
# ---------------------------------------------------------------------------
def _dense_tables(top):
    """Direct-edge tables W (latency) and R (1 - loss) of a dense topology."""
    n = top.n
    W = np.full((n, n), np.inf)
    R = np.zeros((n, n))
    W[top.src, top.dst] = top.latency
    W[top.dst, top.src] = top.latency
    R[top.src, top.dst] = 1.0 - top.loss
    R[top.dst, top.src] = 1.0 - top.loss
    return W, R


def test_c3a_complete_whole_table(E):
    """C3a: complete 20k graph -> every entry is the direct edge
    (_topology_lookupDirectPath, topology.c:1887-1921): lat = 0.0 + w,
    rel = ((1 * a_s) * a_t) * (1 - loss) with a = 1 (no vertex loss).  The
    whole 4e8-entry table against the edge list (the formula itself is
    pinned against the oracle on the shipped topology in test_oracle.py)."""
    top, att = G.make_config("c3a")
    eng = E.Engine(top, att)
    assert eng.is_complete
    eng.compute_all()
    st = eng.stats()
    assert st["mode"] == 2
    assert_fast_path(st, "c3a")
    W, R = _dense_tables(top)
    del top
    n = att.shape[0]
    blk = 1000
    for r0 in range(0, n, blk):
        got = eng.get_rows(r0, blk)
        assert np.array_equal(got["lat"], 0.0 + W[r0:r0 + blk])
        assert np.array_equal(got["rel"], ((1.0 * 1.0) * 1.0) * R[r0:r0 + blk])
        assert np.all(got["hops"] == 1) and np.all(got["flags"] == E.F_DIRECT)
    eng.close()


def test_c3b_dense_minplus(E, oracle_mod):
    """C3b: 20k dense minus one edge (isComplete FALSE -> Dijkstra
    semantics) through the K2 min-plus kernel.  256 rows (both endpoints of
    the removed edge among them) bit-exact against the oracle; every row
    consistent with its chosen predecessors (the reference's left fold);
    the Bellman condition (no arc relaxation shortens the row) on every
    100th row, checked by the oracle's edge-list checker."""
    top, att = G.make_config("c3b")
    W, _ = _dense_tables(top)
    miss = np.argwhere(np.isinf(W) & ~np.eye(top.n, dtype=bool))
    a, b = int(miss[0][0]), int(miss[0][1])
    rng = np.random.default_rng(17)
    sample = np.unique(np.concatenate([[a, b, 0, top.n - 1], rng.choice(top.n, 252, replace=False)]))
    eng = E.Engine(top, att)
    eng.compute_all()
    st = eng.stats()
    assert st["mode"] == 3 and st["rowsComputed"] == top.n
    assert_fast_path(st, "c3b")
    compare_positions(eng, oracle_mod, top, sample, "c3b", block=64)
    np.fill_diagonal(W, np.inf)
    n = top.n
    cols = np.arange(n)
    for r0 in range(0, n, 500):
        blk = eng.get_rows(r0, min(500, n - r0))
        for i in range(blk["lat"].shape[0]):
            s = r0 + i
            lat, hops, pred = blk["lat"][i], blk["hops"][i], blk["pred"][i]
            t = cols[cols != s]
            p = pred[t]
            base = np.where(p == s, 0.0, lat[p])
            assert np.array_equal(lat[t], base + W[p, t]), f"c3b row {s} latency fold"
            assert np.array_equal(hops[t], np.where(p == s, 1, hops[p] + 1)), f"c3b row {s} hops"
    del W
    og = oracle_mod.OracleGraph(top)
    bell = np.arange(0, n, 100)
    for i0 in range(0, bell.shape[0], 50):
        rows = bell[i0:i0 + 50]
        lat = np.concatenate([eng.get_rows(int(r), 1)["lat"] for r in rows])
        viol = og.bellman_violations(att[rows], lat, att, threads=THREADS)
        assert not viol.any(), f"c3b Bellman violations in rows {rows[viol > 0][:5]}"
    eng.close()


@pytest.mark.parametrize("quantum", [0.005, 1.0])
def test_dense_quantized_tie_rows(E, oracle_mod, quantum):
    """Quantised dense graphs (C3b's construction at n = 3,000): 0.005 ms is
    the tie-stress rounding of SURVEY.md §8(d), 1 ms makes equal-distance
    predecessor ties common (like the shipped data's, C1m).  Every tie row
    (F_EXACT) and 256 random rows bit-exact against the oracle's igraph heap
    order; the whole table passes the Bellman check."""
    top = G.dense(3000, seed=3, drop_edge=True, quantum=quantum)
    att = np.arange(top.n, dtype=np.int32)
    eng = E.Engine(top, att)
    eng.compute_all()
    st = eng.stats()
    assert st["mode"] == 3
    assert st["rowsTieRepaired"] == 0, st          # dense tie rows take the full emulation
    ties = tie_positions(eng, E)
    if quantum >= 1.0:
        assert ties.shape[0] > 0 and st["rowsExact"] >= ties.shape[0]
    rng = np.random.default_rng(9)
    pos = np.unique(np.concatenate([ties, rng.choice(eng.T, 256, replace=False)]))
    compare_positions(eng, oracle_mod, top, pos, f"dense q={quantum}", block=128)
    og = oracle_mod.OracleGraph(top)
    for r0 in range(0, eng.T, 500):
        rows = np.arange(r0, min(eng.T, r0 + 500))
        lat = eng.get_rows(r0, rows.shape[0])["lat"]
        assert not og.bellman_violations(att[rows], lat, att, threads=THREADS).any()
    eng.close()
