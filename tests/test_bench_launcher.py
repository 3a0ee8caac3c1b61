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
