"""Drive tools/sim/batch_sim.c on C4 / C5: vertex processings per vertex for
batch orders x bucket widths x per-lane offsets (scheduling probe).

usage: python tools/sim/run_sim.py [c4] [nbatches]
"""
import ctypes
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "shadow-1_amd")]
from shdpe import generators as G  # noqa: E402


class Out(ctypes.Structure):
    _fields_ = [("procs", ctypes.c_double), ("arcs", ctypes.c_double),
                ("phases", ctypes.c_double), ("lanesAct", ctypes.c_double), ("cands", ctypes.c_double),
                ("touched", ctypes.c_double), ("improving", ctypes.c_double), ("laneImp", ctypes.c_double),
                ("skippable", ctypes.c_double), ("skip2", ctypes.c_double),
                ("impv", ctypes.c_double), ("impvMax", ctypes.c_double), ("impvOver", ctypes.c_double * 4)]


def lib():
    so = os.path.join(HERE, "batch_sim.so")
    src = os.path.join(HERE, "batch_sim.c")
    if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
        subprocess.run(["gcc", "-O3", "-march=native", "-shared", "-fPIC", src, "-o", so, "-lm"], check=True)
    L = ctypes.CDLL(so)
    return L


def csr(top):
    import scipy.sparse as sp
    m = top.src != top.dst
    a = np.concatenate([top.src[m], top.dst[m]])
    b = np.concatenate([top.dst[m], top.src[m]])
    w = np.concatenate([top.latency[m], top.latency[m]])
    o = np.lexsort((b, a))
    a, b, w = a[o], b[o], w[o]
    rp = np.zeros(top.n + 1, np.int32)
    np.add.at(rp, a + 1, 1)
    return np.cumsum(rp).astype(np.int32), b.astype(np.int32), w.astype(np.float64)


def bfs_order(rp, col, n):
    from scipy.sparse import csr_matrix
    from scipy.sparse.csgraph import breadth_first_order
    g = csr_matrix((np.ones(col.shape[0]), col, rp), shape=(n, n))
    return breadth_first_order(g, 0, directed=False, return_predecessors=False)


def hub_assign(rp, col, w, n, K):
    """multi-source Dijkstra from the K highest-degree vertices: owner hub and
    distance to it for every vertex"""
    from scipy.sparse import csr_matrix
    from scipy.sparse.csgraph import dijkstra
    deg = np.diff(rp)
    hubs = np.argsort(-deg, kind="stable")[:K]
    g = csr_matrix((w, col, rp), shape=(n, n))
    d, _, src = dijkstra(g, directed=False, indices=hubs, min_only=True, return_predecessors=True)
    return src, d


def run(L, rp, col, w, n, batches, offs, LB, delta, heavy=64, dirty=0, far=0, vkey=None):
    out = Out()
    nb = batches.shape[0] // LB
    rc = L.batch_sim(ctypes.c_int32(n), rp.ctypes.data_as(ctypes.c_void_p),
                     col.ctypes.data_as(ctypes.c_void_p), w.ctypes.data_as(ctypes.c_void_p),
                     batches.ctypes.data_as(ctypes.c_void_p), offs.ctypes.data_as(ctypes.c_void_p),
                     ctypes.c_int32(nb), ctypes.c_int32(LB), ctypes.c_double(delta),
                     ctypes.c_int32(heavy), ctypes.c_int32(dirty), ctypes.c_int32(far), ctypes.byref(out),
                     None if vkey is None else np.ascontiguousarray(vkey, np.float64).ctypes.data_as(ctypes.c_void_p))
    assert rc == 0
    run.cands = out.cands / nb / n
    run.extra = (out.touched / nb / col.shape[0], out.improving / nb / col.shape[0], out.laneImp / nb / n / LB)
    run.skip = (out.skippable / max(out.arcs, 1), out.skip2 / max(out.arcs, 1))
    run.impv = (out.impv / max(out.phases, 1), out.impvMax, [x / max(out.phases, 1) for x in out.impvOver])
    return out.procs / nb / n, out.arcs / nb / col.shape[0], out.phases / nb


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "c4"
    nbs = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    LB = 16
    top, att = G.make_config(wl)
    rp, col, w = csr(top)
    n = top.n
    L = lib()
    mean = w.mean()
    order = bfs_order(rp, col, n)
    rank = np.empty(n, np.int64)
    rank[order] = np.arange(n)
    att_bfs = att[np.argsort(rank[att], kind="stable")]
    K = max(1, min(256, n // 400))
    owner, dh = hub_assign(rp, col, w, n, K)
    att_hub = att[np.lexsort((dh[att], owner[att]))]
    rng = np.random.default_rng(1)
    total_b = att.shape[0] // LB
    pick = np.sort(rng.choice(total_b, nbs, replace=False))
    for oname, seq in (("bfs", att_bfs), ("hub", att_hub)):
        bt = np.concatenate([seq[b * LB:(b + 1) * LB] for b in pick]).astype(np.int32)
        for df in (16, 8, 4, 2, 1):
            for offname in ("none", "hubdist"):
                if offname == "hubdist":
                    offs = dh[bt].astype(np.float64)
                else:
                    offs = np.zeros(bt.shape[0])
                p, a, ph = run(L, rp, col, w, n, bt, offs, LB, df * mean)
                print(f"{wl} order={oname:4s} df={df:3d} off={offname:8s} procs/v={p:5.2f} "
                      f"arcs/m={a:5.2f} phases={ph:6.1f}", flush=True)


if __name__ == "__main__":
    main()
