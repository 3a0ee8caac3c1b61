"""CPU tests of the host side: GraphML reader, generators, the C-ABI library
(loads, exports every symbol of include/shd_pathengine.h, fails loudly with no
GPU), and the N>1 shard/gather logic on gloo."""
import os
import re
import subprocess
import sys

import numpy as np
import pytest

from conftest import GOLDEN, ROOT
from shdpe import generators as G
from shdpe.graph import Topology, read_graphml, write_graphml

HEADER = os.path.join(ROOT, "include", "shd_pathengine.h")


def _declared_symbols():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(shd_(?:pe|topology|graphml|rowstore)_\w+)\s*\(", txt)))


@pytest.fixture(scope="module")
def lib():
    so = os.path.join(ROOT, "shadow-1_amd", "libshdpe.so")
    if not os.path.exists(so):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "shadow-1_amd")], check=True)
    from shdpe import engine
    return engine.load_library()


def test_library_exports_every_declared_symbol(lib):
    syms = _declared_symbols()
    assert len(syms) >= 25
    out = subprocess.run(["nm", "-D", "--defined-only",
                          os.path.join(ROOT, "shadow-1_amd", "libshdpe.so")],
                         capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (\w+)", out))
    missing = [s for s in syms if s not in exported]
    assert not missing, missing
    from shdpe import engine
    assert sorted(engine.EXPORTS) == syms


def test_stats_struct_size_matches_binding(lib):
    """ShdPeStats grows only at its end: the library reports its size (no GPU
    call) and the ctypes mirror must match it field for field."""
    import ctypes
    from shdpe.engine import Stats
    assert lib.shd_pe_stats_size() == ctypes.sizeof(Stats)
    assert Stats._fields_[-1][0] == "relaxCoopAborts"


def test_library_is_gfx950_code_object():
    so = os.path.join(ROOT, "shadow-1_amd", "libshdpe.so")
    data = open(so, "rb").read()
    assert b"gfx950" in data
    assert b"k_sparse_rows" in data and b"k_exact_rows" in data and b"k_direct_rows" in data


def test_engine_fails_loudly_without_gpu(lib):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from shdpe.engine import Engine, EngineError, ENODEV
    top = G.random_sparse(20, 3, seed=1)
    with pytest.raises(EngineError) as ei:
        Engine(top, np.arange(20))
    assert ei.value.code == ENODEV


def test_multigraph_host_build_without_gpu(lib):
    """The host graph build runs before the device check: every multigraph
    is accepted (the create then stops at ENODEV on this GPU-less box) --
    those whose newest parallel edge is a fastest one of its group, those
    whose newest edge (igraph_get_eid's, the one the reference folds) is
    slower than another (round 5: the exact emulation folds that edge's
    latency along the path), and parallel self-loops in any latency order."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from shdpe.engine import Engine, EngineError, ENODEV
    from shdpe.graph import Topology
    base = G.random_sparse(60, 4, seed=2)
    for directed in (False, True):
        b = G.random_sparse(60, 4, seed=2, directed=directed)
        with pytest.raises(EngineError) as ei:
            Engine(G.with_parallel_edges(b, 0.4, seed=3), np.arange(60))
        assert ei.value.code == ENODEV
        with pytest.raises(EngineError) as ei:
            Engine(G.with_parallel_edges(b, 0.4, seed=3, consistent=False, loops=False), np.arange(60))
        assert ei.value.code == ENODEV
        with pytest.raises(EngineError) as ei:
            Engine(G.with_slower_newest_edges(b, 0.4, seed=4), np.arange(60))
        assert ei.value.code == ENODEV
    # two self-loops on vertex 0, the newer one slower: accepted
    top = Topology(base.n, False, np.concatenate([base.src, [0]]), np.concatenate([base.dst, [0]]),
                   np.concatenate([base.latency, [base.latency[base.src == base.dst][0] + 1.0]]),
                   np.concatenate([base.loss, [0.0]]))
    with pytest.raises(EngineError) as ei:
        Engine(top, np.arange(60))
    assert ei.value.code == ENODEV


def test_strerror(lib):
    from shdpe.engine import strerror
    assert "multigraph" in strerror(-6)
    assert strerror(0) == "ok"


def test_graphml_roundtrip():
    top = G.random_sparse(30, 4, seed=3, vloss=True)
    top.ids = ["n%d" % i for i in range(30)]
    back = read_graphml(write_graphml(top))
    assert back.n == top.n and back.m == top.m
    assert np.array_equal(back.src, top.src) and np.array_equal(back.dst, top.dst)
    assert np.array_equal(back.latency, top.latency) and np.array_equal(back.loss, top.loss)
    assert np.array_equal(np.isnan(back.vloss), np.isnan(top.vloss))


def test_graphml_prefers_direct_flag():
    top = G.random_sparse(5, 2, seed=1)
    top.prefers_direct = True
    assert read_graphml(write_graphml(top)).prefers_direct


def test_shipped_fixture_matches_survey():
    top = Topology.load_npz(os.path.join(GOLDEN, "shipped_topology.npz"))
    top.validate()
    assert top.n == 183 and top.m == 16836
    assert np.all(top.loss == 0.005)
    assert np.all(top.vloss == 0.0)
    assert top.latency.min() == 5.0
    assert abs(top.latency.max() - 2293.85) < 1e-9


def test_generators_are_connected_with_self_loops():
    import scipy.sparse as sp
    from scipy.sparse.csgraph import connected_components
    for top in (G.rgg(3000, seed=1), G.power_law(3000, m=3, seed=4),
                G.random_sparse(100, 3, seed=2, directed=True)):
        top.validate()
        loops = top.src == top.dst
        assert np.array_equal(np.sort(top.src[loops]), np.arange(top.n))
        A = sp.coo_matrix((np.ones(top.m), (top.src, top.dst)), shape=(top.n, top.n))
        nc, _ = connected_components(A, directed=top.directed, connection="strong")
        assert nc == 1


def test_config_c2_shape():
    top, att = G.make_config("c2")
    assert top.n == 10_000 and att.shape[0] == 10_000
    nl = top.src != top.dst
    assert 40_000 < int(nl.sum()) < 60_000      # mean degree ~10


def _gloo_worker(rank, world, port, q):
    """Rank `rank` of a world-2 job: its rows come from the engine's own shard
    plan (shd_pe_plan_shards, the function shd_pe_create uses); the blocks
    are assembled the way shd_pe_gather does (one broadcast per shard, each
    landing at its row offset).  No GPU here, so the oracle produces the
    shard's rows -- the GPU engine's sharded tables are checked byte for byte
    in tests/test_gpu_parity.py::test_sharded_engine_*."""
    import torch.distributed as dist
    sys.path[:0] = [os.path.join(ROOT, "shadow-1_amd"), os.path.join(ROOT, "oracle"), ROOT]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import torch

    import oracle as O
    from shdpe.engine import plan_shards
    top = G.random_sparse(120, 4, seed=5)
    att = np.arange(0, 120, 1, dtype=np.int32)
    T = att.shape[0]
    bounds = plan_shards(T, world, unit=16)
    start, count = int(bounds[rank]), int(bounds[rank + 1] - bounds[rank])
    og = O.OracleGraph(top)
    full = torch.zeros(T * T, dtype=torch.float64)
    mine = og.rows(att[start:start + count], att)["lat"]
    full[start * T:(start + count) * T] = torch.from_numpy(mine.ravel())
    for g in range(world):                 # allgatherv = per-shard broadcasts
        lo, hi = int(bounds[g]) * T, int(bounds[g + 1]) * T
        blk = full[lo:hi].clone()
        dist.broadcast(blk, src=g)
        full[lo:hi] = blk
    if rank == 0:
        ref = og.rows(att, att)["lat"]
        q.put(bool(np.array_equal(full.numpy().reshape(T, T).view(np.int64), ref.view(np.int64))))
    dist.barrier()
    dist.destroy_process_group()


def test_shard_and_allgather_world2_gloo(oracle_mod, lib):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + (os.getpid() % 1000)
    procs = [ctx.Process(target=_gloo_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    ok = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
    assert ok


def test_shard_plan(lib):
    """shd_pe_plan_shards: contiguous, covering, unit-aligned, balanced."""
    from shdpe.engine import plan_shards
    for T in (1, 7, 100, 10_000, 16_384, 65_536):
        for world in (1, 2, 3, 8):
            for unit in (1, 16):
                b = plan_shards(T, world, unit)
                assert b[0] == 0 and b[-1] == T and np.all(np.diff(b) >= 0)
                assert np.all(b[:-1] % unit == 0)
                units = np.diff((b + unit - 1) // unit)
                assert units.max() - units.min() <= 1
    assert list(plan_shards(16_384, 8, 16)) == [2048 * g for g in range(9)]


def _fake_table(T, seed=7):
    rng = np.random.default_rng(seed)
    return {"lat": rng.random((T, T)) * 100, "rel": rng.random((T, T)),
            "hops": rng.integers(-1, 30, (T, T)).astype(np.int32),
            "flags": rng.integers(0, 32, (T, T)).astype(np.uint8),
            "pred": rng.integers(-1, 5000, (T, T)).astype(np.int32)}


class _FakeEngine:
    """numpy stand-in with the engine calls shdpe.gather uses (row_checksums,
    get_rows, put_rows, pinned_rows): a rank's table starts with only its own
    block filled; `corrupt` flips one bit of the first foreign row it lands."""

    def __init__(self, T, start, count, corrupt=False):
        from shdpe.engine import row_checksums_host
        self._ck = row_checksums_host
        self.T, self.store_pred, self.corrupt = T, True, corrupt
        full = _fake_table(T)
        self.tab = {k: np.zeros_like(v) for k, v in full.items()}
        for k, v in full.items():
            self.tab[k][start:start + count] = v[start:start + count]

    def row_checksums(self, s, c):
        return self._ck({k: v[s:s + c] for k, v in self.tab.items()})

    def pinned_rows(self, c):
        return {k: np.empty((c,) + v.shape[1:], v.dtype) for k, v in self.tab.items()}

    def get_rows(self, s, c, out):
        for k, v in self.tab.items():
            out[k][:c] = v[s:s + c]

    def put_rows(self, s, rows):
        for k, v in rows.items():
            self.tab[k][s:s + v.shape[0]] = v
        if self.corrupt:
            self.tab["lat"].view(np.uint64)[s, 3] ^= np.uint64(1)
            self.corrupt = False


def _gather_worker(rank, world, port, corrupt_rank, q):
    import torch.distributed as dist
    sys.path[:0] = [os.path.join(ROOT, "shadow-1_amd"), ROOT]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from shdpe.engine import plan_shards
    from shdpe.gather import gather_and_verify
    T = 600
    b = plan_shards(T, world, unit=16)
    start, count = int(b[rank]), int(b[rank + 1] - b[rank])
    eng = _FakeEngine(T, start, count, corrupt=rank == corrupt_rank)
    res = gather_and_verify(eng, dist, rank, world, T, start, count, "host", dist.barrier)
    full = _fake_table(T)
    res["identical"] = all(np.array_equal(eng.tab[k], full[k]) for k in full)
    q.put((rank, res))
    dist.barrier()
    dist.destroy_process_group()


def _run_gather(world, corrupt_rank):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 31500 + (os.getpid() % 1000) + 7 * world + (corrupt_rank + 1)
    procs = [ctx.Process(target=_gather_worker, args=(r, world, port, corrupt_rank, q))
             for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    return out


@pytest.mark.parametrize("world", [2, 3])
def test_gather_verify_host_transport_gloo(lib, world):
    """shdpe.gather on CPU gloo ranks (the bench's N > 1 assembly minus the
    GPU): owners' row fingerprints exchanged, rows moved by host transport,
    every rank's assembled table fingerprinted and compared -- verified, and
    the table equals the union of the owners' blocks."""
    res = _run_gather(world, corrupt_rank=-1)
    for r in range(world):
        assert res[r]["verified"] and res[r]["identical"], res[r]
        assert res[r]["mismatched_rows"] == 0


def test_gather_verify_detects_corruption_gloo(lib):
    """One flipped bit in one landed row on rank 1: rank 1 reports that row,
    and the max-over-ranks count makes rank 0's verdict fail too."""
    res = _run_gather(2, corrupt_rank=1)
    assert res[1]["mismatched_rows"] == 1 and not res[1]["verified"]
    assert res[0]["mismatched_rows"] == 0 and res[0]["mismatched_rows_max_over_ranks"] == 1
    assert not res[0]["verified"]


def test_row_checksums_host_properties(lib):
    """The fingerprint (shd_pe_row_checksums' numpy twin) is a function of
    every field and of each entry's position."""
    from shdpe.engine import row_checksums_host
    t = _fake_table(40)
    base = row_checksums_host(t)
    assert np.unique(base).size == 40
    for k in t:
        u = {kk: vv.copy() for kk, vv in t.items()}
        u[k][5, 7] = u[k][5, 8] if u[k][5, 7] != u[k][5, 8] else u[k][5, 7] + 1
        ck = row_checksums_host(u)
        assert ck[5] != base[5] and np.array_equal(np.delete(ck, 5), np.delete(base, 5)), k
    u = {kk: vv.copy() for kk, vv in t.items()}
    u["lat"][9, [2, 3]] = u["lat"][9, [3, 2]]            # swapped entries
    assert row_checksums_host(u)[9] != base[9]
    nopred = {k: v for k, v in t.items() if k != "pred"}
    assert not np.array_equal(row_checksums_host(nopred), base)
