"""GPU parity at the BASELINE.json configuration sizes, engine sharding, and
concurrent row readers -- all through the C-ABI (libshdpe.so).

Semantics under test: topology.c:1655-1875 (Dijkstra rows: igraph 0.7.1
Dijkstra + _topology_computePathProperties fold) and :1877-1927 (direct rows
of complete graphs).  Bar: lat / rel bit-exact, hops / pred / flags identical
(stricter than north_star's 1e-12 relative); size-independent properties on
top where the oracle cannot cover every row.
"""
import os
import sys
import threading

import numpy as np
import pytest

from shdpe import generators as G
from test_gpu_parity import _assert_rows_equal

pytestmark = pytest.mark.gpu

REL_TOL = 1e-12
THREADS = min(16, os.cpu_count() or 1)


@pytest.fixture(scope="module")
def E():
    from shdpe import engine
    engine.load_library()
    return engine


def _oracle_rows_async(oracle_mod, top, sources, targets):
    """Build the oracle graph and its rows on a host thread (ctypes releases
    the GIL) while the GPU works; join() returns the rows."""
    box = {}

    def run():
        og = oracle_mod.OracleGraph(top)
        box["rows"] = og.rows(sources, targets, threads=THREADS)
        box["og"] = og

    th = threading.Thread(target=run)
    th.start()

    def join():
        th.join()
        return box["rows"], box["og"]
    return join


def _compare_sampled(eng, exp, sources, ctx):
    for i, s in enumerate(sources):
        _assert_rows_equal(eng.get_row(int(s)), {k: v[i] for k, v in exp.items()}, f"{ctx} row {s}")


def _sparse_config(E, oracle_mod, name, n_random=32, every=500):
    """Full-size sparse config: every row computed on the GPU, 32 random rows
    plus every `every`-th row bit-exact against the oracle, and symmetry of
    the latency sub-table over the sampled rows (undirected: d(s,t) = d(t,s)
    up to the rounding of the reversed left fold)."""
    top, att = G.make_config(name)
    rng = np.random.default_rng(11)
    sample = np.unique(np.concatenate([rng.choice(att, n_random, replace=False), att[::every]]))
    join = _oracle_rows_async(oracle_mod, top, sample, att)
    eng = E.Engine(top, att)
    eng.compute_all()
    st = eng.stats()
    assert st["rowsComputed"] == att.shape[0] and st["mode"] == 1
    exp, _ = join()
    _compare_sampled(eng, exp, sample, name)
    # every row of the table is a real Dijkstra row: positive latencies,
    # reliabilities in (0, 1], hops >= 1, no failures (connected, self-loops)
    pos = np.searchsorted(att, sample)
    sub = np.empty((sample.shape[0], sample.shape[0]))
    for i, s in enumerate(sample):
        r = eng.get_row(int(s))
        assert np.all(r["lat"] > 0) and np.all((r["rel"] > 0) & (r["rel"] <= 1))
        assert np.all(r["hops"] >= 1) and not np.any(r["flags"] & 0x03)
        sub[i] = r["lat"][pos]
    assert np.allclose(sub, sub.T, rtol=REL_TOL, atol=0)
    eng.close()
    return st


def test_c4_full_size(E, oracle_mod):
    """C4 (north_star target): BA n=100k, 16,384 attached -- k_batch_rows."""
    st = _sparse_config(E, oracle_mod, "c4")
    assert st["batched"] == 1


def test_c5_full_size(E, oracle_mod):
    """C5: BA n=250k, 65,536 attached (107 GB table on one GPU)."""
    st = _sparse_config(E, oracle_mod, "c5", every=1000)
    assert st["batched"] == 1


def test_c4q_quantised_ties(E, oracle_mod):
    """C4 with latencies rounded to 0.005 ms (like the shipped data): the
    whole table on the GPU; EVERY tie row (found by its F_EXACT flags:
    early-stop emulation + k_tie_write, or cleared by the relevance scan)
    plus 32 random rows bit-exact against the oracle's igraph-heap order."""
    top, att = G.make_config("c4q")
    eng = E.Engine(top, att)
    eng.compute_all()
    st = eng.stats()
    T = eng.T
    tie_pos = []
    for start in range(0, T, 1024):
        blk = eng.get_rows(start, min(1024, T - start))
        tie_pos += list(start + np.flatnonzero((blk["flags"] & E.F_EXACT).any(axis=1)))
        del blk
    assert st["rowsExact"] > 0 and st["rowsTieEarly"] > 0
    # rows the relevance scan cleared keep fast-path parents and no F_EXACT
    assert 0 < len(tie_pos) <= st["rowsExact"]
    rng = np.random.default_rng(3)
    sample = np.unique(np.concatenate([eng.attached[tie_pos], rng.choice(att, 32, replace=False)]))
    exp, _ = _oracle_rows_async(oracle_mod, top, sample, att)()
    _compare_sampled(eng, exp, sample, "c4q")
    eng.close()


def test_c5q_quantised_ties_sampled(E, oracle_mod):
    """C5 with latencies rounded to 0.005 ms: 384 random rows on the GPU
    (tie rows among them take the early-stop path) bit-exact against the
    oracle."""
    top, att = G.make_config("c5q")
    rng = np.random.default_rng(5)
    sample = np.sort(rng.choice(att, 384, replace=False))
    join = _oracle_rows_async(oracle_mod, top, sample, att)
    eng = E.Engine(top, att)
    eng.compute_rows(sample)
    exp, _ = join()
    _compare_sampled(eng, exp, sample, "c5q")
    eng.close()


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


def test_c3a_complete_full_table(E, oracle_mod):
    """C3a: complete 20k graph -> every entry is the direct edge
    (_topology_lookupDirectPath, topology.c:1887-1921): lat = 0.0 + w,
    rel = ((1 * a_s) * a_t) * (1 - loss) with a = 1 (no vertex loss).  The
    whole 4e8-entry table against the edge list (the formula itself is
    pinned against the oracle on the shipped topology in test_oracle.py)."""
    top, att = G.make_config("c3a")
    eng = E.Engine(top, att)
    assert eng.is_complete
    eng.compute_all()
    assert eng.stats()["mode"] == 2
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
    semantics) through the K2 min-plus kernel; 4 rows (incl. both endpoints
    of the removed edge) bit-exact against the oracle, all rows Bellman-
    consistent with their chosen predecessors."""
    top, att = G.make_config("c3b")
    W, _ = _dense_tables(top)
    miss = np.argwhere(np.isinf(W[:, :]) & ~np.eye(top.n, dtype=bool))
    a, b = int(miss[0][0]), int(miss[0][1])
    sample = np.array(sorted({a, b, 0, top.n - 1}), np.int32)
    join = _oracle_rows_async(oracle_mod, top, sample, att)
    eng = E.Engine(top, att)
    eng.compute_all()
    st = eng.stats()
    assert st["mode"] == 3 and st["rowsComputed"] == top.n
    exp, _ = join()
    _compare_sampled(eng, exp, sample, "c3b")
    # predecessor consistency on a sweep of rows: lat[t] == lat[pred] + w
    # bit-exact (the reference's left fold), hops[t] == hops[pred] + 1
    np.fill_diagonal(W, np.inf)
    for s in range(0, top.n, 5000):
        r = eng.get_row(s)
        lat, hops, pred = r["lat"], r["hops"], r["pred"]
        t = np.flatnonzero(np.arange(top.n) != s)
        p = pred[t]
        base = np.where(p == s, 0.0, lat[p])
        assert np.array_equal(lat[t], base + W[p, t])
        assert np.array_equal(hops[t], np.where(p == s, 1, hops[p] + 1))
        # no shorter relaxation through any vertex u (lat[t] <= lat[u] + w)
        lu = lat.copy()
        lu[s] = 0.0
        for t0 in range(0, top.n, 2000):
            tt = np.arange(t0, min(top.n, t0 + 2000))
            cand = (lu[:, None] + W[:, tt]).min(axis=0)
            keep = tt != s
            assert np.all(lat[tt][keep] <= cand[keep])
    eng.close()


# ---------------------------------------------------------------------------
# multi-GPU: row shards
# ---------------------------------------------------------------------------
FIELDS = ("lat", "rel", "hops", "pred", "flags")


def _all_rows(eng):
    return eng.get_rows(0, eng.T)


def _same(a, b, ctx):
    for k in FIELDS:
        assert np.array_equal(a[k].view(np.uint8), b[k].view(np.uint8)), (ctx, k)


def _shard_case(name):
    if name == "batched":
        top = G.power_law(20_000, m=3, seed=41)
        return top, G.sample_attached(top.n, 1000, seed=3), 5
    if name == "sparse":
        top = G.rgg(3000, seed=42)
        return top, np.arange(top.n, dtype=np.int32), 0
    if name == "dense":
        return G.dense(600, seed=43, drop_edge=True), np.arange(600, dtype=np.int32), 0
    top = G.power_law(2000, m=2, seed=44, quantum=1.0)        # tie rows (k_exact_rows)
    return top, np.arange(top.n, dtype=np.int32), 0


@pytest.mark.parametrize("name", ["batched", "sparse", "dense", "ties"])
@pytest.mark.parametrize("nshards", [2, 3])
def test_sharded_engine_matches_single(E, name, nshards):
    """nDevices logical shards on the one test GPU: each shard computes its
    own contiguous rows on its own stream / host thread; rows read before
    the gather come from the owning shard, after shd_pe_gather from the
    assembled table -- byte-identical to the 1-shard engine either way."""
    top, att, force = _shard_case(name)
    one = E.Engine(top, att, force_mode=force)
    one.compute_all()
    ref = _all_rows(one)
    st1 = one.stats()
    one.close()
    eng = E.Engine(top, att, force_mode=force, devices=[0] * nshards)
    b = eng.shard_bounds()
    assert b.shape[0] == nshards + 1 and b[0] == 0 and b[-1] == eng.T
    assert eng.owned == (0, eng.T)
    eng.compute_all()
    st = eng.stats()
    assert st["nShards"] == nshards and st["rowsComputed"] == eng.T
    assert st["rowsExact"] == st1["rowsExact"]
    _same(_all_rows(eng), ref, f"{name} per-shard")
    eng.gather()
    _same(_all_rows(eng), ref, f"{name} gathered")
    eng.close()


def test_multiprocess_shard_engines(E):
    """shardIndex / shardCount: each engine owns one contiguous block of the
    plan and computes only that; together they are the 1-engine table.
    Reading another engine's row needs the gather (SHD_PE_ENOTOWNED), and
    the gather needs the cross-process communicator (SHD_PE_ECOMM)."""
    top, att, force = _shard_case("batched")
    one = E.Engine(top, att, force_mode=force)
    one.compute_all()
    ref = _all_rows(one)
    one.close()
    engs = [E.Engine(top, att, force_mode=force, shard_index=i, shard_count=2) for i in range(2)]
    (s0, c0), (s1, c1) = engs[0].owned, engs[1].owned
    assert s0 == 0 and s0 + c0 == s1 and s1 + c1 == engs[0].T
    assert list(engs[0].shard_bounds()) == [0, s1, s1 + c1]
    for e in engs:
        e.compute_all()
        s, c = e.owned
        got = e.get_rows(s, c)
        for k in FIELDS:
            assert np.array_equal(got[k], ref[k][s:s + c]), k
    with pytest.raises(E.EngineError) as ei:
        engs[0].get_row(int(engs[0].attached[s1]))
    assert ei.value.code == E.ENOTOWNED
    with pytest.raises(E.EngineError) as ei:
        engs[0].gather()
    assert ei.value.code == E.ECOMM
    for e in engs:
        e.close()


def test_c4_two_shards_full_size(E):
    """C4 in two logical shards (LB and batch plan per shard) == one shard."""
    top, att = G.make_config("c4")
    one = E.Engine(top, att)
    one.compute_all()
    two = E.Engine(top, att, devices=[0, 0])
    two.compute_all()
    rng = np.random.default_rng(5)
    for p in np.sort(rng.choice(att.shape[0], 48, replace=False)):
        a, b = one.get_rows(int(p), 1), two.get_rows(int(p), 1)
        _same(a, b, f"c4 row {p}")
    one.close()
    two.close()


# ---------------------------------------------------------------------------
# concurrent readers (header: get_row may be called from any thread)
# ---------------------------------------------------------------------------
def test_get_row_from_8_threads(E):
    """8 host threads call shd_pe_get_row on overlapping sources before any
    compute: rows are computed on demand under the engine mutex, the
    computed-row flags are acquire/release atomics; every result equals a
    serial engine's row."""
    top = G.rgg(2000, seed=61)
    att = np.arange(top.n, dtype=np.int32)
    ref = E.Engine(top, att)
    ref.compute_all()
    serial = _all_rows(ref)
    ref.close()
    eng = E.Engine(top, att)
    rng = np.random.default_rng(7)
    picks = [rng.choice(att, 60) for _ in range(8)]
    errors = []

    def reader(k):
        try:
            for s in picks[k]:
                r = eng.get_row(int(s))
                p = int(s)
                for f in FIELDS:
                    if not np.array_equal(r[f], serial[f][p]):
                        errors.append((k, p, f))
        except Exception as ex:          # noqa: BLE001 - reported below
            errors.append((k, repr(ex)))

    th = [threading.Thread(target=reader, args=(k,)) for k in range(8)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors[:5]
    eng.close()


_RANK_SCRIPT = r"""
import os, sys
import numpy as np
root = sys.argv[1]
sys.path[:0] = [os.path.join(root, "shadow-1_amd")]
import torch
import torch.distributed as dist
from shdpe import generators as G
from shdpe.engine import Engine
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dist.init_process_group("gloo", rank=rank, world_size=world)
top = G.power_law(20_000, m=3, seed=41)
att = G.sample_attached(top.n, 1000, seed=3)
eng = Engine(top, att, device=0, force_mode=5, shard_index=rank, shard_count=world)
eng.compute_all()
s0, cnt = eng.owned
rows = eng.get_rows(s0, cnt)
T = eng.T
out = {}
for k in ("lat", "rel", "hops", "pred", "flags"):
    blk = torch.from_numpy(np.ascontiguousarray(rows[k]).view(np.uint8).reshape(-1).copy())
    sizes = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(sizes, torch.tensor([blk.numel()], dtype=torch.int64))
    mx = int(max(s.item() for s in sizes))
    pad = torch.zeros(mx, dtype=torch.uint8)
    pad[:blk.numel()] = blk
    parts = [torch.zeros(mx, dtype=torch.uint8) for _ in range(world)]
    dist.all_gather(parts, pad)
    out[k] = np.concatenate([p[:int(s.item())].numpy() for p, s in zip(parts, sizes)])
if rank == 0:
    np.savez(sys.argv[2], **out)
dist.barrier()
eng.close()
dist.destroy_process_group()
"""


def test_two_rank_processes_gloo_gather_match_single_engine(E, tmp_path):
    """Two rank processes on the test GPU (what bench.py --gpus 2 runs, one
    engine per rank with shardIndex / shardCount), their row blocks exchanged
    over gloo (all fields): the assembled table is byte-identical to one
    engine's.  The ranks share one GPU here, so the exchange cannot be RCCL
    (one device per rank); the engine-owned RCCL gather is covered by the
    in-process multi-shard tests above."""
    import socket
    import subprocess
    top, att, force = _shard_case("batched")
    one = E.Engine(top, att, force_mode=force)
    one.compute_all()
    ref = _all_rows(one)
    one.close()
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    out = str(tmp_path / "table.npz")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-c", _RANK_SCRIPT, root, out], env=env))
    for p in procs:
        assert p.wait(timeout=240) == 0
    got = np.load(out)
    for k in FIELDS:
        assert np.array_equal(got[k], ref[k].view(np.uint8).reshape(-1)), k
