"""Benchmark: path-table construction (source rows/sec), BASELINE.json metric.

python bench.py --gpus N --steps K --warmup W [--workload c4] [--no-allgather]

A step = one full path-table construction for the workload (all S source
rows, S = T = attached vertices).  With N ranks (one process per GPU,
torchrun) every rank builds ONE engine for its own GPU with
shardIndex = rank, shardCount = N: the engine's shard plan
(shd_pe_shard_bounds) gives it a contiguous block of rows with an equal
number of kernel work units, and it computes only those (strong scaling: the
table is fixed, ranks split it; no exchange on the data path).
With N > 1 the whole table is then assembled on every GPU through the
engine-owned RCCL communicator (shd_pe_comm_init + shd_pe_gather: one
ncclAllGather per field over xGMI) and VERIFIED: the owners' per-row 64-bit
fingerprints taken before the exchange must equal every rank's fingerprints
of its assembled table (shdpe/gather.py).  Timed separately, never part of
`value`, reported under "allgather"; the line is always emitted, and the exit
status is 0 only for a verified assembly (4 mismatch, 5 RCCL / engine error,
6 watchdog timeout).  At N > 1 `per_rank` carries every rank's step, kernel
and exact-kernel time, roofline fraction and rows (min / mean / max and the
slowest rank), so a scaling line shows where the max-over-ranks time goes.  One-GPU
rehearsal (BENCH_REHEARSE_ONE_GPU=1, ranks share cuda:0, RCCL refuses such a
communicator) moves the rows over gloo + shd_pe_put_rows instead.

Default workload: C4 (BASELINE.json configs[3], the north_star target:
100k-vertex power-law topology, 16,384 attached sources).  Inputs (graph,
attached set) are uploaded before the timed region; rows stay in HBM (the
D2H to the host path cache is outside `value`).

rank 0 prints ONE JSON line.  cpu_baseline = the oracle (C restatement of
igraph 0.7.1 Dijkstra + topology.c fold) on 1 host thread, on a bounded
sample of the same rows (the reference serialises all Dijkstra runs under
graphLock, topology.c:1747-1781).  --tie-stress adds the 0.005-quantised
variants (c2q, c4q: SURVEY.md §8d) with their tie-row counts.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "shadow-1_amd"), os.path.join(ROOT, "oracle")]

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X spec (MI355X_MICROARCH.md)
FP64_VALU_PEAK_TF = 78.6       # MI355X FP64 vector spec


def algorithmic_bytes_per_row(n, m_arcs, T):
    """SURVEY.md §8(d) frozen formula for a sparse row: 12*m_arcs + 12*n + 20*T."""
    return 12 * m_arcs + 12 * n + 20 * T


def cpu_baseline(top, att, budget_s=12.0, max_rows=4000, threads=1):
    """Time the oracle on a bounded sample of the workload's rows.

    threads=1 matches the reference (graphLock serialises every Dijkstra,
    topology.c:1747-1781); threads>1 is the generous all-cores CPU bound of
    SURVEY.md §8(d), one source row per thread."""
    import oracle as O
    O.build()
    og = O.OracleGraph(top)
    rng = np.random.default_rng(0)
    order = rng.permutation(att.shape[0])
    done, t0 = 0, time.perf_counter()
    chunk = threads                  # grows while rows are cheap (dense rows take seconds)
    while done < max_rows and time.perf_counter() - t0 < budget_s:
        c0 = time.perf_counter()
        srcs = att[order[done:done + chunk]]
        if srcs.shape[0] == 0:
            break
        og.rows(srcs, att, threads=threads)
        done += srcs.shape[0]
        if time.perf_counter() - c0 < 0.25 * budget_s / 8:
            chunk = min(chunk * 2, 64 * threads)
    dt = time.perf_counter() - t0
    extra = {}
    if threads == 1 and done:
        # Dijkstra alone (no fold / row build), same rows: SURVEY.md §8(d)
        # asks for the split; the fold + row is the difference
        k, d0 = 0, time.perf_counter()
        while k < done and time.perf_counter() - d0 < budget_s / 4:
            og.raw(int(att[order[k]]), att)
            k += 1
        extra = {"dijkstra_only_rows_per_s": k / (time.perf_counter() - d0),
                 "dijkstra_only_rows": k}
    return {"value": done / dt, "unit": "source rows/s", "cores": threads, "kind": "port", **extra,
            "sample": f"{done} random source rows of the same workload (all {att.shape[0]} "
                      f"targets each), igraph-0.7.1-faithful 2-wheap Dijkstra + "
                      f"_topology_computePathProperties fold, {threads} thread(s), {dt:.1f} s"}


def load_traffic(workload):
    """PMC traffic of the dominant kernel (profiles/traffic_<wl>.json, made by
    tools/traffic_json.py) -- only if it was measured on a library built from
    the same kernel sources as this one; a stale capture is dropped."""
    from shdpe.engine import kernel_source_hash
    p = os.path.join(ROOT, "profiles", f"traffic_{workload}.json")
    if os.path.exists(p):
        with open(p) as f:
            t = json.load(f)
        if t.get("src_hash") == kernel_source_hash():
            return t
    return None


def roofline_of(st, n, m_arcs, T, count):
    """Roofline of the dominant kernel from the engine's own HIP-event kernel
    times (stats), algorithmic work per SURVEY.md §8(d): sparse rows
    12*m_arcs + 12*n + 20*T bytes each (HBM), direct rows 36*T bytes each
    (HBM), dense min-plus 2 flops per executed relaxation (FP64 VALU)."""
    ms_kernel = st["msSparseKernel"] + st["msDirectKernel"] + st["msDenseKernel"]
    launches = max(1, st["launchesSparse"] + st["launchesDirect"] + st["launchesDense"])
    avg_launch_ms = ms_kernel / launches
    bound, unit, peak = "hbm", "GB/s", HBM_PEAK_GBS
    if st["mode"] == 2:
        work = 36 * T * count
        kname = "k_direct_rows"
        achieved = work / (avg_launch_ms * 1e-3) / 1e9
    elif st["mode"] == 3:
        # dense min-plus: SURVEY §8d prices a sweep at 2*n^2 flops per row;
        # sweeps skip K chunks that cannot improve (chunk epochs), so the
        # work counted is what the kernels executed: visited (row tile, K
        # chunk) pairs x 2 flops per relaxation, + the pred pass
        work = st["denseFlops"] / max(1, st["launchesDense"])
        kname = "k_minplus"
        bound, unit, peak = "valu-fp64", "TFLOP/s", FP64_VALU_PEAK_TF
        achieved = work / (avg_launch_ms * 1e-3) / 1e12
    else:
        work = algorithmic_bytes_per_row(n, m_arcs, T) * count
        kname = "k_batch_rows" if st["batched"] else "k_sparse_rows"
        achieved = work / (avg_launch_ms * 1e-3) / 1e9
    return {"bound": bound, "kernel": kname, "achieved": achieved, "peak": peak, "unit": unit,
            "frac": achieved / peak, "algorithmic_per_launch": work,
            "avg_launch_ms": avg_launch_ms, "launches": launches}


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv):
    """--gpus N > 1 without a launcher: start N fresh rank processes of this
    script (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in their env), before
    this process touches the GPU or torch.cuda.  Rank 0's stdout (the JSON
    line) is relayed; the first child to fail takes the others down and its
    exit code is returned.  No exec: the children are ordinary subprocesses."""
    import signal
    import subprocess
    import threading
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + argv,
                                      env=env, stdout=subprocess.PIPE if r == 0 else None))

    def relay(p):
        for line in iter(p.stdout.readline, b""):
            sys.stdout.write(line.decode(errors="replace"))
            sys.stdout.flush()
    th = threading.Thread(target=relay, args=(procs[0],), daemon=True)
    th.start()
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            c = p.poll()
            if c is None:
                continue
            live.remove(p)
            if c != 0 and rc == 0:
                rc = c if c > 0 else 128 - c
                sys.stderr.write(f"bench.py: rank {procs.index(p)} exited with {c}; stopping the others\n")
                for q in live:
                    q.send_signal(signal.SIGTERM)
        if live:
            time.sleep(0.2)
            if rc:
                t0 = time.time()
                while any(q.poll() is None for q in live) and time.time() - t0 < 20:
                    time.sleep(0.2)
                for q in live:
                    if q.poll() is None:
                        q.kill()
                for q in live:
                    q.wait()
                live = []
    th.join(timeout=10)
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one process per GPU); without a launcher's WORLD_SIZE this "
                         "process starts the N rank processes itself")
    ap.add_argument("--dry-launch", action="store_true",
                    help="launcher self-test: every rank prints its rank env as JSON and exits")
    ap.add_argument("--secondary", default="c1,c2,c3a,c3b,c5",
                    help="comma list of further configs timed after the headline (rank 0, N=1; "
                         "'' = off): ms_per_step, rows/s and roofline of each")
    ap.add_argument("--host-fill", type=int, default=1,
                    help="time the end-to-end host fill (compute + rows into pinned buffers + "
                         "shd_rowstore_store_row for every row) once after the timed region")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="c4")
    ap.add_argument("--allgather", action="store_true", help="(default with --gpus > 1; kept for old scripts)")
    ap.add_argument("--no-allgather", action="store_true",
                    help="N > 1: skip the verified table assembly after the timed region")
    ap.add_argument("--gather-timeout", type=float, default=300.0,
                    help="seconds before a hung assembly is reported (error in the line) and the "
                         "ranks exit")
    ap.add_argument("--sub-shards", type=int, default=1,
                    help="row shards per GPU, computed concurrently on their own streams")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--cpu-threads", type=int, default=min(16, os.cpu_count() or 1),
                    help="threads of the all-cores CPU bound (1 = skip; the GPU box's "
                         "share is 16 CPUs, os.cpu_count() there shows the whole machine)")
    ap.add_argument("--no-stream", action="store_true",
                    help="skip the device-copy HBM bandwidth reference")
    ap.add_argument("--tie-stress", default="c2q,c4q,c5q,c3bq",
                    help="comma list of quantised variants timed after the headline (rank 0, "
                         "N=1; '' = off): their tie-row fraction and k_exact_rows time")
    ap.add_argument("--d2h-rows", type=int, default=2048,
                    help="rows copied to host buffers through shd_pe_get_row after the timed "
                         "region (PCIe-inclusive rate, reported separately; 0 = off)")
    args = ap.parse_args()

    if args.gpus < 1:
        sys.exit("bench.py: --gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        sys.stderr.write(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}: refusing to "
                         f"report a {world}-rank run as {args.gpus} GPUs\n")
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # stdout carries exactly one line, rank 0's JSON: whatever the libraries
    # print there (gloo's connection notices, RCCL) goes to stderr instead
    out_fd = os.dup(1)
    sys.stdout.flush()
    os.dup2(2, 1)
    emit = (lambda line: os.write(out_fd, (line + "\n").encode())) if rank == 0 else (lambda line: None)
    if args.dry_launch:
        if os.environ.get("BENCH_DRY_NOISE"):
            os.write(1, b"[Gloo] Rank is connected to 1 peer ranks\n")   # a library's stdout chatter
        os.write(out_fd, (json.dumps({"rank": rank, "local_rank": local, "world": world,
                                      "master": f"{os.environ.get('MASTER_ADDR')}:"
                                                f"{os.environ.get('MASTER_PORT')}",
                                      "pid": os.getpid()}) + "\n").encode())   # one write
        # launcher self-test hooks: one rank fails, the others hang
        if os.environ.get("BENCH_DRY_FAIL_RANK") == str(rank):
            sys.exit(3)
        if os.environ.get("BENCH_DRY_FAIL_RANK"):
            time.sleep(120)
        return
    dist = None
    # BENCH_REHEARSE_ONE_GPU=1: rehearse the N-rank flow on a one-GPU box
    # (every rank's shard engine on cuda:0, gloo for the barrier and the
    # max-over-ranks reduction); the driver's multi-GPU runs use RCCL
    rehearse = os.environ.get("BENCH_REHEARSE_ONE_GPU") == "1"
    if world > 1:
        import torch
        import torch.distributed as dist
        if rehearse:
            local = 0
            dist.init_process_group("gloo")
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from shdpe import generators as G
    from shdpe.engine import Engine, DEBUG_ENV

    # SHDPE_* tuning variables reach the library only through its debug flag
    dbg = DEBUG_ENV if any(k.startswith("SHDPE_") for k in os.environ) else 0
    top, att = G.make_config(args.workload)
    eng = Engine(top, att, device=local, shard_index=rank, shard_count=world, debug_flags=dbg,
                 devices=[local] * args.sub_shards if args.sub_shards > 1 else None)
    T = eng.T
    start, count = eng.owned
    st0 = eng.stats()
    n, m_arcs = st0["nVertices"], st0["nArcs"]

    def barrier_sync():
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            dist.barrier()
        eng.synchronize()

    # setup (untimed): pick the faster k_batch_rows variant on this box
    # (shd_pe_tune computes the shard twice per variant; no-op off the batched
    # path), then the warm-up steps
    eng.tune()
    for _ in range(args.warmup):
        eng.compute_all()
    barrier_sync()
    eng.reset_stats()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.compute_all()
    eng.synchronize()
    barrier_sync()
    elapsed = time.perf_counter() - t0
    st = eng.stats()
    rl = roofline_of(st, n, m_arcs, T, count)
    per_rank = None
    if dist is not None:
        import torch
        dev = "cpu" if rehearse else f"cuda:{local}"
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        # every rank's own numbers, so a scaling line shows which rank and
        # which kernel sets the max-over-ranks time
        per_rank = collect_per_rank(dist, dev, world, rank_record(st, elapsed, args.steps, count, rl))
        elapsed = float(t.item())

    rows_total = T * args.steps
    value = rows_total / elapsed
    bound, bytes_per_launch, achieved, avg_launch_ms = (rl["bound"], rl["algorithmic_per_launch"],
                                                        rl["achieved"], rl["avg_launch_ms"])
    traffic = load_traffic(args.workload)
    traffic_bytes = (traffic or {}).get("bytes_per_launch")
    if traffic_bytes and count != T:
        # the PMC capture is of the whole table on one GPU; a shard's launch
        # moves its share (per-row traffic is uniform across batches)
        traffic_bytes = traffic_bytes * count / T
    out = {
        "metric": "path-table source rows/sec (latency+reliability)",
        "value": value,
        "unit": "source rows/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic",
        "config": {"workload": args.workload, "desc": G.CONFIGS.get(args.workload, {}).get("desc"),
                   "vertices": n, "arcs": m_arcs,
                   "sources": T, "targets": T, "rows_per_step": T,
                   "parallelism": f"source-row shards x{world}"},
        "edges_relaxed_per_s": m_arcs * rows_total / elapsed,
        "roofline": dict(rl, traffic=traffic_bytes, traffic_tag=(traffic or {}).get("tag")),
        "rows_exact": st["rowsExact"] // max(1, args.steps),
        "tie_row_fraction": st["rowsExact"] / max(1, args.steps * count),
        "ms_exact_per_step": st["msExactKernel"] / max(1, args.steps),
        "batch_kernel_waves": st["batchWaves"] or None,
        "batch_lanes": st["batchLanes"] or None,
        "batch_post_kernel_waves": st["batchPostWaves"] or None,
    }
    if per_rank is not None:
        out["per_rank"] = per_rank
    # ---- N > 1: the shared table assembled on every rank and verified
    # (untimed, never in `value`); a watchdog reports a hung exchange in the
    # line instead of leaving the driver without one ----
    import threading
    emitted = threading.Lock()
    done = threading.Event()

    def emit_once(o):
        if emitted.acquire(blocking=False):
            emit(json.dumps(o))

    gather_res = None
    if world > 1 and not args.no_allgather:
        from shdpe.gather import gather_and_verify

        def on_timeout():
            if done.is_set():
                return
            o = dict(out, allgather={"verified": False, "transport": "rehearse-host" if rehearse else "rccl",
                                     "error": f"no completion within {args.gather_timeout:.0f} s"})
            sys.stderr.write(f"bench.py: rank {rank}: table assembly timed out\n")
            emit_once(o)
            # the value stands and the line says the table was not assembled;
            # the exit status says so too (only a verified assembly exits 0)
            os._exit(EXIT_ASSEMBLY_TIMEOUT)
        wd = threading.Timer(args.gather_timeout, on_timeout)
        wd.daemon = True
        wd.start()
        row_bytes = T * (8 + 8 + 4 + 1 + (4 if eng.store_pred else 0))
        try:
            gather_res = gather_and_verify(eng, dist, rank, world, T, start, count,
                                           "host" if rehearse else "rccl", barrier_sync,
                                           reduce_device=None if rehearse else f"cuda:{local}",
                                           row_bytes=row_bytes)
        except Exception as e:       # an RCCL / engine error: reported, value stands
            gather_res = {"verified": False, "transport": "host" if rehearse else "rccl",
                          "error": f"{type(e).__name__}: {e}"}
        wd.cancel()
        gather_res["fields"] = "lat f64, rel f64, hops i32, flags u8" + (", pred i32" if eng.store_pred else "")
        out["allgather"] = gather_res
    d2h = None
    if args.d2h_rows > 0 and count > 0:
        # PCIe-inclusive: the shard's rows into host buffers after the timed
        # region, (a) page-locked buffers from shd_pe_host_alloc (DMA lands in
        # place), (b) fresh pageable numpy arrays (pinned staging + threaded
        # host copy; includes first-touch page faults)
        k = min(args.d2h_rows, count)
        row_bytes = T * (8 + 8 + 4 + 1 + (4 if eng.store_pred else 0))
        eng.get_rows(start, min(k, 8))
        pin = eng.pinned_rows(k)
        eng.get_rows(start, k, out=pin)          # warm (maps the pinned pages on the device)
        d0 = time.perf_counter()
        eng.get_rows(start, k, out=pin)
        dt = time.perf_counter() - d0
        del pin
        p0 = time.perf_counter()
        eng.get_rows(start, k)
        dtp = time.perf_counter() - p0
        d2h = {"rows": int(k), "ms_per_row": dt / k * 1e3, "GB/s": k * row_bytes / dt / 1e9,
               "pageable_GB/s": k * row_bytes / dtp / 1e9,
               "pcie_inclusive_rows_per_s": 1.0 / (elapsed / args.steps / count + dt / k),
               "note": "shd_pe_get_rows after the timed region (not in value): GB/s into "
                       "shd_pe_host_alloc buffers; pageable_GB/s into fresh numpy arrays"}

    if rank == 0 and not args.no_stream:
        sbw = eng.stream_bandwidth()     # 16-B streaming copy kernel, same device
        out["roofline"]["stream_GBps"] = sbw
        if bound == "hbm":
            out["roofline"]["frac_of_stream"] = achieved / sbw
            tb = out["roofline"]["traffic"]
            if tb:
                # measured L2-miss bytes (PMC, profiles/traffic_<wl>.json) over
                # this run's launch time: how close the kernel runs to the
                # bandwidth it actually moves
                out["roofline"]["traffic_GBps"] = tb / (avg_launch_ms * 1e-3) / 1e9
                out["roofline"]["traffic_frac_of_stream"] = out["roofline"]["traffic_GBps"] / sbw
                out["roofline"]["traffic_over_algorithmic"] = tb / bytes_per_launch
    if d2h:
        out["d2h"] = d2h
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(top, att, budget_s=args.cpu_budget)
        out["speedup_vs_cpu"] = value / out["cpu_baseline"]["value"]
        if args.cpu_threads > 1:
            allc = cpu_baseline(top, att, budget_s=args.cpu_budget / 2, threads=args.cpu_threads)
            out["cpu_baseline_all_cores"] = allc
            out["speedup_vs_cpu_all_cores"] = value / allc["value"]
    if rank == 0 and world == 1 and args.host_fill:
        out["host_fill"] = host_fill(eng, top)
    eng.close()
    if rank == 0 and world == 1 and args.host_fill:
        host_fill_image(out["host_fill"], top, att, dbg)
    if rank == 0 and world == 1 and args.secondary:
        out["secondary"] = [secondary(wl, args.steps, dbg) for wl in args.secondary.split(",") if wl]
    if rank == 0 and world == 1 and args.tie_stress:
        out["tie_stress"] = [tie_stress(wl, args.steps, dbg) for wl in args.tie_stress.split(",") if wl]
    done.set()
    emit_once(out)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    rc = assembly_exit_code(gather_res)
    if rc:
        sys.stderr.write(f"bench.py: rank {rank}: table assembly not verified (exit {rc}): "
                         f"{json.dumps(gather_res)}\n")
        sys.exit(rc)


EXIT_ASSEMBLY_MISMATCH = 4     # assembled rows differ from the owners' fingerprints
EXIT_ASSEMBLY_ERROR = 5        # RCCL / engine error, or no verdict
EXIT_ASSEMBLY_TIMEOUT = 6      # the watchdog fired (hung exchange)


def assembly_exit_code(gather_res):
    """0 only for a verified table assembly (or none attempted); the JSON line
    is emitted first either way, so the measured value is never lost."""
    if gather_res is None:
        return 0
    if gather_res.get("mismatched_rows_max_over_ranks", 0) > 0:
        return EXIT_ASSEMBLY_MISMATCH
    if gather_res.get("error") or gather_res.get("verified") is not True:
        return EXIT_ASSEMBLY_ERROR
    return 0


RANK_FIELDS = ("elapsed_ms_per_step", "kernel_ms_per_step", "exact_ms_per_step", "frac", "rows",
               "rows_exact")


def rank_record(st, elapsed, steps, count, rl):
    """This rank's numbers for the per-rank block (floats, RANK_FIELDS order)."""
    k = max(1, steps)
    kern = st["msSparseKernel"] + st["msDirectKernel"] + st["msDenseKernel"]
    return [elapsed / k * 1e3, kern / k, st["msExactKernel"] / k, rl["frac"], float(count),
            float(st["rowsExact"] // k)]


def collect_per_rank(dist, dev, world, record):
    """All-gather every rank's rank_record (one small float64 tensor per rank
    over the job's process group) and summarise; every rank gets the block."""
    import torch
    mine = torch.tensor(record, dtype=torch.float64, device=dev)
    allr = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(allr, mine)
    return per_rank_summary([a.cpu().tolist() for a in allr])


def per_rank_summary(records):
    """N > 1: every rank's step time, kernel time (HIP events on its stream),
    exact-kernel time, roofline fraction and row count, plus min / mean / max
    of the step and kernel times and the rank that set the max."""
    ranks = [dict(zip(RANK_FIELDS, r), rank=i) for i, r in enumerate(records)]
    for r in ranks:
        r["rows"] = int(r["rows"])
        r["rows_exact"] = int(r["rows_exact"])
    out = {"ranks": ranks}
    for f in ("elapsed_ms_per_step", "kernel_ms_per_step", "frac"):
        v = [r[f] for r in ranks]
        out[f] = {"min": min(v), "mean": sum(v) / len(v), "max": max(v)}
    out["slowest_rank"] = max(ranks, key=lambda r: r["elapsed_ms_per_step"])["rank"]
    out["kernel_max_over_mean"] = (out["kernel_ms_per_step"]["max"] /
                                   max(1e-12, out["kernel_ms_per_step"]["mean"]))
    return out


def secondary(workload, steps, dbg):
    """Another BASELINE config timed the same way as the headline (setup and
    tune untimed, rows resident in HBM): ms per full table, rows/s and the
    roofline of its dominant kernel (C3a: k_direct_rows, HBM; C5:
    k_batch_rows, HBM; C3b: k_minplus, FP64 VALU)."""
    from shdpe import generators as G
    from shdpe.engine import Engine
    g0 = time.perf_counter()
    top, att = G.make_config(workload)
    eng = Engine(top, att, debug_flags=dbg)
    setup_s = time.perf_counter() - g0
    st0 = eng.stats()
    eng.tune()
    eng.compute_all()                        # warm-up
    eng.synchronize()
    eng.reset_stats()
    # small tables (C1: 183 rows, C2) get more steps: their table takes
    # milliseconds, and one step would be mostly launch overhead noise
    k = max(1, min(steps, 3 if eng.T > 12_000 else 20))
    t0 = time.perf_counter()
    for _ in range(k):
        eng.compute_all()
    eng.synchronize()
    el = (time.perf_counter() - t0) / k
    st = eng.stats()
    T = eng.T
    out = {"workload": workload, "desc": G.CONFIGS.get(workload, {}).get("desc"),
           "vertices": st0["nVertices"], "arcs": st0["nArcs"], "rows": int(T), "steps": k,
           "ms_per_step": el * 1e3, "rows_per_s": T / el,
           "edges_relaxed_per_s": st0["nArcs"] * T / el,
           "roofline": roofline_of(st, st0["nVertices"], st0["nArcs"], T, T),
           "tie_rows": st["rowsExact"] // k, "ms_exact_per_step": st["msExactKernel"] / k,
           "batch_lanes": st["batchLanes"] or None, "setup_s": setup_s}
    tr = load_traffic(workload)
    if tr and tr.get("bytes_per_launch"):
        # PMC capture of this config's dominant kernel (same kernel sources)
        rl = out["roofline"]
        rl["traffic"] = tr["bytes_per_launch"]
        rl["traffic_tag"] = tr.get("tag")
        if rl["bound"] == "hbm":
            rl["traffic_over_algorithmic"] = tr["bytes_per_launch"] / rl["algorithmic_per_launch"]
            rl["traffic_GBps"] = tr["bytes_per_launch"] / (rl["avg_launch_ms"] * 1e-3) / 1e9
    eng.close()
    return out


def host_fill(eng, top, block=1024, threads=0):
    """End-to-end path-cache fill as the drop-in does it (topology.c:1805-1864
    for every row), outside `value`, two ways:
    (1) shd_pe_fill_rowstore on a fresh engine (host_fill_image below): the
        call computes the table while a host thread prepares the page-locked
        image, then the device packs the row store's triangular image (17 B
        per unordered pair) and one DMA lands it in the memory the store
        adopts -- the headline `end_to_end_over_compute`;
    (2) here, after one more compute_all: rows DMA'd in blocks into
        page-locked buffers (shd_pe_get_rows) and stored with
        shd_rowstore_store_rows, the next block's copy overlapping the
        current block's store (`rows_path`)."""
    import threading
    from shdpe.engine import RowStore
    T = eng.T
    start, count = eng.owned
    eng.synchronize()
    t0 = time.perf_counter()
    eng.compute_all()
    eng.synchronize()
    t_gpu = time.perf_counter() - t0
    store = RowStore(top.n, eng.attached)
    fields = ("lat", "rel", "flags")
    bufs = [eng.pinned_rows(min(block, count), fields) for _ in range(2)]
    blocks = [(b0, min(block, count - b0)) for b0 in range(0, count, block)]
    d2h_s, store_s = [0.0], 0.0
    res = []

    def fetch(i, buf):
        b0, c = blocks[i]
        f0 = time.perf_counter()
        eng.get_rows(start + b0, c, out=buf)
        d2h_s[0] += time.perf_counter() - f0

    f0 = time.perf_counter()
    th = threading.Thread(target=fetch, args=(0, bufs[0]))
    th.start()
    for i, (b0, c) in enumerate(blocks):
        th.join()
        if i + 1 < len(blocks):
            th = threading.Thread(target=fetch, args=(i + 1, bufs[(i + 1) % 2]))
            th.start()
        b = bufs[i % 2]
        s0 = time.perf_counter()
        res.append(store.store_rows(eng.attached[start + b0:start + b0 + c], b["lat"], b["rel"],
                                    b["flags"], threads=threads))
        store_s += time.perf_counter() - s0
    fill_s = time.perf_counter() - f0
    rows_path = {"block_rows": block, "ms_fill": fill_s * 1e3, "ms_d2h_sum": d2h_s[0] * 1e3,
                 "ms_store_sum": store_s * 1e3, "host_fill_rows_per_s": count / (t_gpu + fill_s),
                 "end_to_end_over_compute": (t_gpu + fill_s) / t_gpu,
                 "entries_stored": int(store.size()), "store_GB": store.memory_bytes() / 1e9,
                 "rows_all_success": int(sum(int(r.sum()) for r in res)),
                 "how": "shd_pe_get_rows into shd_pe_host_alloc buffers (lat, rel, flags) + "
                        "shd_rowstore_store_rows (threads by slot rows), copy of block b+1 "
                        "overlapping the store of block b"}
    out = {"rows": int(count), "ms_compute": t_gpu * 1e3, "rows_path": rows_path}
    store.close()
    del bufs
    return out


def host_fill_image(out, top, att, dbg):
    """The drop-in's one call on a freshly built engine (graph upload
    untimed; no variant pick -- the drop-in computes once, so its first
    compute runs the default variant and allocates its scratch inside the
    timed call): shd_pe_fill_rowstore computes every row, with the host image
    prepared on a host thread meanwhile, packs and DMAs it.  The ratio is that
    call's wall time over the tuned compute_all's (`ms_compute`, same box)."""
    from shdpe.engine import Engine, RowStore
    eng = Engine(top, att, debug_flags=dbg)
    eng.synchronize()
    img = RowStore(top.n, eng.attached)
    i0 = time.perf_counter()
    ok, ms = eng.fill_rowstore(img)
    t_img = time.perf_counter() - i0
    t_gpu = out["ms_compute"] * 1e-3
    out.update({"ms_fill": t_img * 1e3, "ms_compute_and_image_prep": ms["alloc"], "ms_pack": ms["pack"],
                "ms_dma": ms["dma"], "image_GB": img.memory_bytes() / 1e9,
                "entries_stored": int(img.size()), "rows_all_success": int(ok.sum()),
                "host_fill_rows_per_s": out["rows"] / t_img,
                "end_to_end_over_compute": t_img / t_gpu,
                "how": "fresh engine, one shd_pe_fill_rowstore call: compute_all on the device while a "
                       "host thread maps, first-touches (16 threads, huge pages) and registers the "
                       "image; device pack of the triangular cache image; one DMA into it; the row "
                       "store adopts it"})
    assert out["rows_path"]["entries_stored"] == out["entries_stored"], out
    img.close()
    eng.close()


def tie_stress(workload, steps, dbg):
    """Quantised variant (latencies rounded to 0.005 ms, like the shipped data):
    rows whose equal-distance predecessor ties go to k_exact_rows."""
    from shdpe import generators as G
    from shdpe.engine import Engine
    top, att = G.make_config(workload)
    eng = Engine(top, att, debug_flags=dbg)
    eng.tune()
    eng.compute_all()                        # warm-up
    eng.reset_stats()
    t0 = time.perf_counter()
    k = max(1, min(steps, 2))
    for _ in range(k):
        eng.compute_all()
    eng.synchronize()
    el = (time.perf_counter() - t0) / k
    st = eng.stats()
    eng.close()
    return {"workload": workload, "rows": int(eng.T), "ms_per_step": el * 1e3,
            "rows_per_s": eng.T / el, "tie_rows": st["rowsExact"] // k,
            "tie_row_fraction": st["rowsExact"] / k / eng.T,
            "tie_rows_early_stop": st["rowsTieEarly"] // k,
            "ms_exact_kernel_per_step": st["msExactKernel"] / k,
            "ms_main_kernel_per_step": (st["msSparseKernel"] + st["msDenseKernel"]) / k}


if __name__ == "__main__":
    main()
