"""Multi-rank table assembly with verification.

One process per GPU, each engine owning a contiguous block of table rows
(shardIndex / shardCount).  After the compute, every rank assembles the whole
T x T table -- the shared path table that replaces the reference's one-row-
at-a-time Dijkstra under graphLock (topology.c:1747-1781) -- and proves the
assembled copy identical to what the owners computed:

  1. each rank fingerprints its own rows on its device (shd_pe_row_checksums,
     one 64-bit checksum per row) BEFORE the exchange;
  2. the fingerprints are all-gathered over torch.distributed (a few KB);
  3. the table moves: RCCL over xGMI (shd_pe_comm_init + shd_pe_gather: one
     ncclAllGather per field) -- or, where RCCL has no communicator (several
     ranks sharing one GPU in a rehearsal), host transport: each owner's rows
     go out in chunks over torch.distributed broadcasts and land through
     shd_pe_put_rows;
  4. every rank fingerprints all T rows of its assembled table and compares;
     the mismatch count is max-reduced so every rank reaches the same verdict.

The engine argument is duck-typed (row_checksums, get_rows, put_rows,
pinned_rows, gather, comm_init): tests drive the same code with a numpy
stand-in on CPU gloo ranks (tests/test_host.py).
"""
from __future__ import annotations

import time

import numpy as np

FIELDS = ("lat", "rel", "hops", "flags", "pred")


def exchange_checksums(dist, start: int, count: int, own: np.ndarray, T: int) -> np.ndarray:
    """All-gather every rank's (start, count, checksums); the expected
    fingerprint of each of the T rows.  Raises if the blocks do not tile
    [0, T) exactly once."""
    parts = [None] * dist.get_world_size()
    dist.all_gather_object(parts, (int(start), int(count), np.asarray(own, np.uint64).tobytes()))
    expect = np.zeros(T, np.uint64)
    seen = np.zeros(T, np.int32)
    for s0, c0, b in parts:
        expect[s0:s0 + c0] = np.frombuffer(b, np.uint64)
        seen[s0:s0 + c0] += 1
    if not np.all(seen == 1):
        raise RuntimeError("row blocks of the ranks do not tile the table exactly once")
    return expect, [(s0, c0) for s0, c0, _ in parts]


def compare_checksums(dist, expect: np.ndarray, full: np.ndarray, reduce_device=None) -> dict:
    """Mismatching rows here, and the max over ranks (every rank agrees)."""
    import torch
    bad = np.flatnonzero(np.asarray(full, np.uint64) != expect)
    t = torch.tensor([bad.size], dtype=torch.int64,
                     device=reduce_device if reduce_device is not None else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    worst = int(t.item())
    return {"verified": worst == 0, "mismatched_rows": int(bad.size),
            "mismatched_rows_max_over_ranks": worst, "first_bad_rows": bad[:8].tolist()}


def host_transport(eng, dist, rank: int, blocks, T: int, chunk: int = 256) -> int:
    """Every owner's rows to every other rank over torch.distributed
    broadcasts, chunk by chunk, landing through eng.put_rows.  Returns the
    bytes this rank received."""
    import torch
    bufs = eng.pinned_rows(chunk)
    fields = [k for k in FIELDS if bufs.get(k) is not None]
    got = 0
    for r, (s0, c0) in enumerate(blocks):
        for b0 in range(0, c0, chunk):
            c = min(chunk, c0 - b0)
            if rank == r:
                eng.get_rows(s0 + b0, c, out=bufs)
            for k in fields:
                dist.broadcast(torch.from_numpy(bufs[k][:c]), src=r)
            if rank != r:
                eng.put_rows(s0 + b0, {k: bufs[k][:c] for k in fields})
                got += sum(bufs[k][:c].nbytes for k in fields)
    return got


def gather_and_verify(eng, dist, rank: int, world: int, T: int, start: int, count: int,
                      transport: str, barrier, reduce_device=None, row_bytes: int = 0) -> dict:
    """Steps 1-4 above.  transport: "rccl" (shd_pe_comm_init + shd_pe_gather)
    or "host" (torch.distributed broadcasts + shd_pe_put_rows)."""
    c0 = time.perf_counter()
    own = eng.row_checksums(start, count)
    ck_own_ms = (time.perf_counter() - c0) * 1e3
    expect, blocks = exchange_checksums(dist, start, count, own, T)
    if transport == "rccl":
        from shdpe.engine import Engine
        uid = [Engine.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        eng.comm_init(uid[0])
    barrier()
    g0 = time.perf_counter()
    if transport == "rccl":
        eng.gather()
        received = (T - count) * row_bytes
        how = ("shd_pe_gather: RCCL over xGMI, one ncclAllGather per field (equal row blocks; "
               "a broadcast group otherwise) into each rank's full table")
    else:
        received = host_transport(eng, dist, rank, blocks, T)
        how = ("host transport: owners' rows broadcast over torch.distributed (gloo) in 256-row "
               "chunks, landed with shd_pe_put_rows (ranks share a GPU: RCCL has no communicator)")
    barrier()
    ms = (time.perf_counter() - g0) * 1e3
    c1 = time.perf_counter()
    full = eng.row_checksums(0, T)
    ck_full_ms = (time.perf_counter() - c1) * 1e3
    res = {"transport": transport, "ms": ms, "bytes_received_per_rank": int(received),
           "GBps_received_per_rank": received / max(ms, 1e-9) / 1e6,
           "checksum_own_rows_ms": ck_own_ms, "checksum_all_rows_ms": ck_full_ms, "how": how}
    res.update(compare_checksums(dist, expect, full, reduce_device))
    res["check"] = ("per-row 64-bit fingerprints (shd_pe_row_checksums, all fields) of the owners' "
                    "rows before the exchange == fingerprints of all T rows of this rank's "
                    "assembled table after it")
    return res
