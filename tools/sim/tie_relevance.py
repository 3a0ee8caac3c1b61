"""How far must the igraph heap emulation of a tie row run?  (CPU analysis,
oracle-backed: tools only.)

For every row of a config, from the oracle's igraph Dijkstra (final
distances of the popped vertices, pop order):
  * ambiguous entries, as k_batch_rows marks them: the tight in-arcs with the
    minimum dist[u] are not exactly one, or that minimum equals dist[v]
    (zero-increment arc); mt(v) = that minimum (the tied predecessor distance);
  * the fast-path parent chain of every target, up to the first ambiguous
    vertex it meets (a tie row = some target meets one);
  * thr_all = max mt over every ambiguous entry (what the export sends today),
    thr_rel = max mt over the ambiguous entries FIRST met on a target chain;
  * pops the early-stop emulation needs under each threshold.
Usage: python tools/sim/tie_relevance.py c4q [procs]"""
import os
import sys
from multiprocessing import Pool

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "shadow-1_amd"), ROOT]

from shdpe import generators as G  # noqa: E402
from oracle import oracle as O     # noqa: E402

_st = {}


def _init(name):
    top, att = G.make_config(name)
    _st["top"], _st["att"] = top, att
    _st["og"] = O.OracleGraph(top)
    s, d, w = top.src.astype(np.int64), top.dst.astype(np.int64), top.latency
    if top.directed:
        U, V, W = s, d, w
    else:
        U, V, W = np.concatenate([s, d]), np.concatenate([d, s]), np.concatenate([w, w])
    _st["arcs"] = (U, V, W)


def _row(i):
    top, att, og = _st["top"], _st["att"], _st["og"]
    U, V, W = _st["arcs"]
    src = int(att[i])
    dist, _par, order = og.raw(src, att)
    n = top.n
    popped = np.zeros(n, bool)
    popped[order] = True
    ok = popped[U] & popped[V]
    du = np.where(ok, dist[U], np.inf)
    tight = ok & (du + W == dist[V]) & (du <= dist[V])
    tu, tv = U[tight], V[tight]
    tdu = du[tight]
    mt = np.full(n, np.inf)
    np.minimum.at(mt, tv, tdu)
    atmin = tdu == mt[tv]
    cnt = np.bincount(tv[atmin], minlength=n)
    fp = np.full(n, -1, np.int64)
    fp[tv[atmin]] = tu[atmin]
    has = np.isfinite(mt)
    amb = has & ((cnt != 1) | (mt == dist)) & (np.arange(n) != src)
    if not amb.any():
        return None
    # fast chains of every target up to the first ambiguous vertex
    x = att.astype(np.int64).copy()
    x = x[x != src]
    first = np.full(x.shape[0], -1, np.int64)
    live = np.ones(x.shape[0], bool)
    for _ in range(n):
        hit = live & amb[x]
        first[hit] = x[hit]
        live &= ~hit & (x != src) & (fp[x] >= 0)
        if not live.any():
            break
        x = np.where(live, fp[x], x)
    rel = first[first >= 0]
    if rel.shape[0] == 0:
        return (i, int(amb.sum()), 0, float(mt[amb].max()), -1.0, len(order), 0, 0)
    thr_all = float(mt[amb].max())
    thr_rel = float(mt[np.unique(rel)].max())
    keys = dist[order]
    pops_all = int(np.searchsorted(np.maximum.accumulate(keys), thr_all, side="right"))
    pops_rel = int(np.searchsorted(np.maximum.accumulate(keys), thr_rel, side="right"))
    return (i, int(amb.sum()), int(np.unique(rel).shape[0]), thr_all, thr_rel, len(order),
            pops_all, pops_rel)


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "c4q"
    procs = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    limit = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    _, att = G.make_config(name)
    rows = range(att.shape[0] if not limit else min(limit, att.shape[0]))
    out = []
    with Pool(procs, initializer=_init, initargs=(name,)) as p:
        for r in p.imap_unordered(_row, rows, chunksize=16):
            if r is not None:
                out.append(r)
    out.sort()
    print(f"{name}: {len(out)} rows with ambiguous entries")
    print("row   amb  relAmb      thr_all      thr_rel  popped  pops_all  pops_rel")
    tot_a = tot_r = 0
    for r in out:
        if r[2] == 0:
            continue
        print("%5d %5d %6d %12.4f %12.4f %7d %9d %9d" % r)
        tot_a += r[6]
        tot_r += r[7]
    print(f"tie rows (a target chain meets an ambiguous entry): {sum(1 for r in out if r[2])}; "
          f"pops total all={tot_a} rel={tot_r}; worst all={max((r[6] for r in out), default=0)} "
          f"rel={max((r[7] for r in out), default=0)}")


if __name__ == "__main__":
    main()
