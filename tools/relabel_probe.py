"""Probe: does vertex numbering change k_batch_rows time?

Permutes the C4 (or C5) topology's vertex ids with several orders and times
compute_all on each (results are the same paths under other ids; only the
memory layout of the [v][LB] scratch and the CSR changes).  Scheduling probe,
not a parity test.

usage: python tools/relabel_probe.py [c4|c5] [orders...]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "shadow-1_amd")]

from shdpe import generators as G  # noqa: E402
from shdpe.graph import Topology  # noqa: E402
from shdpe.engine import Engine  # noqa: E402


def csr(top):
    import scipy.sparse as sp
    m = top.src != top.dst
    a, b = top.src[m], top.dst[m]
    g = sp.coo_matrix((np.ones(a.shape[0]), (a, b)), shape=(top.n, top.n)).tocsr()
    return (g + g.T).tocsr()


def csr_w(top):
    import scipy.sparse as sp
    m = top.src != top.dst
    a, b, w = top.src[m], top.dst[m], top.latency[m]
    g = sp.coo_matrix((w, (a, b)), shape=(top.n, top.n)).tocsr()
    return (g + g.T).tocsr()


def order_of(top, kind):
    n = top.n
    if kind == "identity":
        return np.arange(n)
    if kind == "random":
        return np.random.default_rng(0).permutation(n)
    g = csr(top)
    deg = np.diff(g.indptr)
    if kind == "degree":
        return np.argsort(-deg, kind="stable")
    if kind == "bfs":
        from scipy.sparse.csgraph import breadth_first_order
        o = breadth_first_order(g, int(np.argmax(deg)), directed=False, return_predecessors=False)
        return o
    if kind == "hubdist":
        from scipy.sparse.csgraph import dijkstra
        w = csr_w(top)
        d = dijkstra(w, directed=False, indices=int(np.argmax(deg)))
        return np.argsort(d, kind="stable")
    if kind == "rcm":
        from scipy.sparse.csgraph import reverse_cuthill_mckee
        return reverse_cuthill_mckee(g, symmetric_mode=True)
    raise KeyError(kind)


def relabel(top, att, order):
    """order[k] = old id of new vertex k."""
    new_of = np.empty(top.n, np.int64)
    new_of[order] = np.arange(top.n)
    t2 = Topology(n=top.n, directed=top.directed, src=new_of[top.src], dst=new_of[top.dst],
                  latency=top.latency, loss=top.loss,
                  vloss=None if top.vloss is None else top.vloss[order], name=top.name + "_rl")
    return t2, np.sort(new_of[att]).astype(np.int32)


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "c4"
    kinds = sys.argv[2:] or ["identity", "random", "degree", "bfs", "rcm", "hubdist"]
    top, att = G.make_config(wl)
    for kind in kinds:
        t2, a2 = relabel(top, att, order_of(top, kind))
        eng = Engine(t2, a2)
        eng.compute_all()
        eng.reset_stats()
        t0 = time.perf_counter()
        for _ in range(3):
            eng.compute_all()
        eng.synchronize()
        dt = (time.perf_counter() - t0) / 3
        st = eng.stats()
        print(f"{wl} {kind:9s} {dt * 1e3:8.1f} ms/table  kernel {st['msSparseKernel'] / 3:8.1f} ms", flush=True)
        eng.close()


if __name__ == "__main__":
    main()
