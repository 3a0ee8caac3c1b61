"""Row shards of one path table, and concurrent row readers,
through the C-ABI (libshdpe.so).

What runs where:
  * logical shards on the one test GPU (devices=[0]*N): per-shard streams and
    host threads, gather by device copies -- byte-identical to one engine;
  * shardIndex / shardCount engines (one per process in Shadow / bench.py),
    their blocks exchanged over gloo by two rank processes sharing the GPU;
  * the RCCL gathers (in-process ncclCommInitAll over distinct devices, and
    the cross-process communicator of shd_pe_comm_init) need one device per
    rank: test_rccl_gather_distinct_devices runs only when >= 2 GPUs are
    visible and is skipped on the 1-GPU test box; the cross-process calls
    (ncclCommInitRank, the per-field ncclAllGather group) run on one GPU
    through a one-rank communicator (test_rccl_one_rank_communicator_gather),
    the multi-rank exchange itself is NOT verified on hardware by this suite.
"""
import os
import sys
import threading

import numpy as np
import pytest

from shdpe import generators as G

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def E():
    from shdpe import engine
    engine.load_library()
    return engine


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


def _same_blocks(a_eng, b_eng, ctx, block=1024):
    """Whole tables byte-identical, all five fields, in row blocks."""
    T = a_eng.T
    for p0 in range(0, T, block):
        c = min(block, T - p0)
        _same(a_eng.get_rows(p0, c), b_eng.get_rows(p0, c), f"{ctx} rows {p0}..{p0 + c}")


@pytest.fixture(scope="module")
def c4_one(E):
    """The 1-shard C4 engine (headline config), computed once for the
    full-size shard tests; its device fingerprints equal the numpy twin's."""
    top, att = G.make_config("c4")
    one = E.Engine(top, att)
    one.tune()
    one.compute_all()
    ck = one.row_checksums(0, one.T)
    probe = one.get_rows(0, 64)
    assert np.array_equal(ck[:64], E.row_checksums_host(probe))
    yield top, att, one, ck
    one.close()


def test_c4_two_shards_full_size(E, c4_one):
    """C4 in two logical shards (LB 16, batch plan per shard) == one shard,
    whole table, all fields."""
    top, att, one, ck = c4_one
    two = E.Engine(top, att, devices=[0, 0])
    two.compute_all()
    _same_blocks(one, two, "c4 x2")
    assert np.array_equal(two.row_checksums(0, two.T), ck)
    two.close()


@pytest.mark.parametrize("wpe", ["tune", "4", "8", "coop"])
def test_c4_eight_shards_full_size(E, c4_one, monkeypatch, wpe):
    """C4 in eight logical shards = what each rank of the 8-GPU run computes
    (2,048 rows, LB 8 batches, the tune's variant pick -- and each of the two
    variants forced, and the cooperative relax forced: two workgroups of one
    XCD per batch): whole table byte-identical to one engine's, before and
    after the gather, and the device fingerprints agree."""
    top, att, one, ck = c4_one
    dbg = 0
    if wpe == "coop":
        monkeypatch.setenv("SHDPE_BATCH_COOP", "2")
        dbg = E.DEBUG_ENV
    elif wpe != "tune":
        monkeypatch.setenv("SHDPE_BATCH_WPE", wpe)
        dbg = E.DEBUG_ENV
    eng = E.Engine(top, att, devices=[0] * 8, debug_flags=dbg)
    assert list(eng.shard_bounds()) == [2048 * g for g in range(9)]
    if wpe == "tune":
        eng.tune()
    eng.reset_stats()
    eng.compute_all()
    st = eng.stats()
    assert st["batched"] == 1 and st["batchLanes"] == 8 and st["rowsExact"] == 0, st
    assert st["rowsTieRepaired"] == 0 and st["relaxCoopAborts"] == 0, st
    if wpe == "coop":
        assert st["batchCoop"] == 2, st
    elif wpe != "tune":
        assert st["batchWaves"] == int(wpe) and st["batchCoop"] == 0
    _same_blocks(one, eng, f"c4 x8 wpe {wpe}")
    eng.gather()
    assert np.array_equal(eng.row_checksums(0, eng.T), ck)
    eng.close()


def test_put_rows_host_transport_and_checksums(E):
    """Two shardIndex / shardCount engines (one per rank in bench.py's
    one-GPU rehearsal): fingerprints of the owners' blocks == the 1-engine
    table's; each engine lands the other's rows through shd_pe_put_rows
    (host transport) and then reads the whole table byte-identical to one
    engine, with matching device fingerprints.  Own rows are refused."""
    top, att, force = _shard_case("batched")
    one = E.Engine(top, att, force_mode=force)
    one.compute_all()
    ref = _all_rows(one)
    ref_ck = one.row_checksums(0, one.T)
    assert np.array_equal(ref_ck, E.row_checksums_host(ref))
    one.close()
    engs = [E.Engine(top, att, force_mode=force, shard_index=i, shard_count=2) for i in range(2)]
    for e in engs:
        e.compute_all()
    own = np.concatenate([e.row_checksums(*e.owned) for e in engs])
    assert np.array_equal(own, ref_ck)
    for a, b in ((0, 1), (1, 0)):
        s, c = engs[b].owned
        half = c // 2                     # two puts: the table is assembled on the second
        engs[a].put_rows(s, engs[b].get_rows(s, half))
        engs[a].put_rows(s, engs[b].get_rows(s, half))     # a repeated block counts once
        with pytest.raises(E.EngineError) as ei:
            engs[a].get_rows(s + half, c - half)
        assert ei.value.code == E.ENOTOWNED
        engs[a].put_rows(s + half, engs[b].get_rows(s + half, c - half))
    for e in engs:
        _same(_all_rows(e), ref, "put_rows assembled")
        assert np.array_equal(e.row_checksums(0, e.T), ref_ck)
    s, c = engs[0].owned
    with pytest.raises(E.EngineError) as ei:
        engs[0].put_rows(s, {k: v[s:s + 1] for k, v in ref.items()})
    assert ei.value.code == E.EINVAL
    for e in engs:
        e.close()


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


def _visible_gpus():
    try:
        import torch
        return torch.cuda.device_count()
    except Exception:          # noqa: BLE001 - no torch / no ROCm runtime
        return 0


def test_rccl_one_rank_communicator_gather(E):
    """The cross-process RCCL path on one GPU: a one-rank communicator
    (shd_pe_comm_unique_id + shd_pe_comm_init with shardCount 1) makes
    shd_pe_gather issue the calls an N-rank run does (ncclCommInitRank, a
    group of one ncclAllGather per field, in place); every field is still
    byte-identical to an engine that never gathered, and the gather was
    timed (it ran)."""
    top, att, force = _shard_case("batched")
    one = E.Engine(top, att, force_mode=force)
    one.compute_all()
    ref = _all_rows(one)
    one.close()
    eng = E.Engine(top, att, force_mode=force, shard_index=0, shard_count=1)
    eng.comm_init(E.Engine.comm_unique_id())
    eng.compute_all()
    eng.gather()
    _same(_all_rows(eng), ref, "rccl one-rank gathered")
    st = eng.stats()
    assert st["nShards"] == 1 and st["msGather"] > 0, st
    eng.close()


def test_rccl_gather_distinct_devices(E):
    """Two shards on two distinct devices inside one engine: shd_pe_gather
    builds an ncclCommInitAll communicator and assembles the table with a
    group of per-shard broadcasts over xGMI; every device's gathered table
    is byte-identical to the 1-GPU engine's.  Skipped with < 2 GPUs."""
    if _visible_gpus() < 2:
        pytest.skip("RCCL gather needs >= 2 GPUs (one device per rank)")
    top, att, force = _shard_case("batched")
    one = E.Engine(top, att, force_mode=force)
    one.compute_all()
    ref = _all_rows(one)
    one.close()
    eng = E.Engine(top, att, force_mode=force, devices=[0, 1])
    eng.compute_all()
    eng.gather()
    _same(_all_rows(eng), ref, "rccl gathered")
    st = eng.stats()
    assert st["nShards"] == 2 and st["msGather"] > 0
    eng.close()
