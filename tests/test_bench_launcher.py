"""bench.py --gpus N without a launcher starts N fresh rank processes itself
(before any GPU call), relays rank 0's line, propagates a failing rank's
exit code, and refuses a --gpus / WORLD_SIZE mismatch (CPU only: the
--dry-launch children report their rank env and exit)."""
import json
import os
import subprocess
import sys
import time

from conftest import ROOT

BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None, timeout=60):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True,
                          timeout=timeout, env=env)


def test_launcher_spawns_n_ranks():
    r = _run(["--gpus", "4", "--dry-launch"])
    assert r.returncode == 0, r.stderr
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert sorted(x["rank"] for x in lines) == [0, 1, 2, 3]
    assert all(x["world"] == 4 and x["local_rank"] == x["rank"] for x in lines)
    assert len({x["master"] for x in lines}) == 1 and lines[0]["master"].startswith("127.0.0.1:")
    assert len({x["pid"] for x in lines}) == 4


def test_single_gpu_runs_in_process():
    r = _run(["--gpus", "1", "--dry-launch"])
    assert r.returncode == 0
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1 and lines[0]["world"] == 1


def test_world_size_mismatch_is_an_error():
    r = _run(["--gpus", "8", "--dry-launch"], {"WORLD_SIZE": "2", "RANK": "0"})
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr
    r = _run(["--gpus", "2", "--dry-launch"], {"WORLD_SIZE": "2", "RANK": "1"})
    assert r.returncode == 0


def test_failing_rank_stops_the_others():
    t0 = time.time()
    r = _run(["--gpus", "3", "--dry-launch"], {"BENCH_DRY_FAIL_RANK": "2"}, timeout=90)
    assert r.returncode == 3, (r.returncode, r.stderr)
    assert "rank 2 exited with 3" in r.stderr
    assert time.time() - t0 < 60          # the sleeping ranks were terminated


def test_library_stdout_chatter_goes_to_stderr():
    """Only JSON on stdout: a library printing to fd 1 in a rank (gloo does)
    lands on stderr."""
    r = _run(["--gpus", "2", "--dry-launch"], {"BENCH_DRY_NOISE": "1"})
    assert r.returncode == 0
    out = [x for x in r.stdout.splitlines() if x.strip()]
    assert len(out) == 2 and all(x.startswith("{") for x in out), r.stdout
    assert "[Gloo]" in r.stderr


# ---- N > 1 line shape: per-rank block and the exit status of the assembly ----
def _import_bench():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", BENCH)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _fake_stats(kernel_ms, exact_ms, rows_exact, steps):
    return {"msSparseKernel": kernel_ms * steps, "msDirectKernel": 0.0, "msDenseKernel": 0.0,
            "msExactKernel": exact_ms * steps, "rowsExact": rows_exact * steps}


def _per_rank_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    bench = _import_bench()
    dist.init_process_group("gloo", rank=rank, world_size=world)
    steps = 4
    st = _fake_stats(10.0 + 2 * rank, 0.5 * rank, rank, steps)
    rl = {"frac": 0.1 + 0.01 * rank}
    rec = bench.rank_record(st, (11.0 + 2 * rank) * steps * 1e-3, steps, 2048 + rank, rl)
    q.put((rank, bench.collect_per_rank(dist, "cpu", world, rec)))
    dist.barrier()
    dist.destroy_process_group()


def test_per_rank_block_world3_gloo():
    """What rank 0 puts under `per_rank` at N > 1: every rank's step / kernel
    / exact time, frac and rows, min / mean / max and the slowest rank --
    gathered over a real 3-rank gloo group (the GPU runs use RCCL)."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29700 + (os.getpid() % 500)
    world = 3
    procs = [ctx.Process(target=_per_rank_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    blk = got[0]
    assert all(got[r] == blk for r in range(world))          # every rank holds the same block
    ranks = blk["ranks"]
    assert [r["rank"] for r in ranks] == [0, 1, 2]
    for r in ranks:
        i = r["rank"]
        assert abs(r["elapsed_ms_per_step"] - (11.0 + 2 * i)) < 1e-9
        assert abs(r["kernel_ms_per_step"] - (10.0 + 2 * i)) < 1e-9
        assert abs(r["exact_ms_per_step"] - 0.5 * i) < 1e-9
        assert abs(r["frac"] - (0.1 + 0.01 * i)) < 1e-12
        assert r["rows"] == 2048 + i and r["rows_exact"] == i
    assert blk["slowest_rank"] == 2
    assert blk["elapsed_ms_per_step"] == {"min": 11.0, "mean": 13.0, "max": 15.0}
    assert abs(blk["kernel_max_over_mean"] - 14.0 / 12.0) < 1e-12
    json.dumps(blk)                                           # it goes into the JSON line


def test_assembly_exit_codes():
    """Only a verified assembly (or none) exits 0; the line is emitted first."""
    bench = _import_bench()
    assert bench.assembly_exit_code(None) == 0
    assert bench.assembly_exit_code({"verified": True, "mismatched_rows_max_over_ranks": 0}) == 0
    assert bench.assembly_exit_code({"verified": False, "mismatched_rows_max_over_ranks": 3}) == 4
    assert bench.assembly_exit_code({"verified": False, "error": "RuntimeError: x"}) == 5
    assert bench.assembly_exit_code({"transport": "rccl"}) == 5        # no verdict
    assert bench.EXIT_ASSEMBLY_TIMEOUT == 6
