"""Dense min-plus path (K2): parity vs oracle and timing."""
import os, sys, time
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(R, "shadow-1_amd"), os.path.join(R, "oracle")]
import numpy as np
from shdpe import generators as G
from shdpe.graph import Topology
from shdpe.engine import Engine
from oracle import OracleGraph

def check(top, att, srcs, tag):
    t0 = time.time(); eng = Engine(top, att); tc = time.time() - t0
    st0 = eng.stats()
    t0 = time.time(); eng.compute_rows(srcs); dt = time.time() - t0
    st = eng.stats()
    og = OracleGraph(top)
    bad = 0
    for s in srcs[:min(len(srcs), int(os.environ.get("QCHK", "64")))]:
        g = eng.get_row(int(s)); o = og.row(int(s), eng.attached)
        ok = (np.array_equal(g['lat'].view(np.int64), o['lat'].view(np.int64)) and np.array_equal(g['rel'].view(np.int64), o['rel'].view(np.int64))
              and np.array_equal(g['hops'], o['hops']) and np.array_equal(g['pred'], o['pred']))
        if not ok:
            bad += 1
            if bad <= 2:
                k = np.flatnonzero((g['lat'] != o['lat']) | (g['rel'] != o['rel']) | (g['hops'] != o['hops']) | (g['pred'] != o['pred']))
                print(tag, "row", s, "bad cols", k[:4], g['lat'][k[:2]], o['lat'][k[:2]], g['hops'][k[:2]], o['hops'][k[:2]], g['pred'][k[:2]], o['pred'][k[:2]], flush=True)
    print(f"{tag}: n={top.n} mode={st['mode']} create={tc:.1f}s rows={len(srcs)} wall={dt:.3f}s dense_ms={st['msDenseKernel']:.1f} sweeps={st['denseSweeps']} exact_rows={st['rowsExact']} exact_ms={st['msExactKernel']:.1f} bad={bad}", flush=True)
    eng.close()

shipped = Topology.load_npz(os.path.join(R, "tests/golden/shipped_topology.npz"))
m1 = G.minus_one_edge(shipped, seed=3)
check(m1, np.arange(183), np.arange(183, dtype=np.int32), "shipped-1")
d = G.dense(1500, seed=3, drop_edge=True)
check(d, np.arange(1500), np.arange(0, 1500, 7, dtype=np.int32), "dense1500")
d = G.dense(int(os.environ.get("QN", "6000")), seed=3, drop_edge=True)
att = np.arange(d.n, dtype=np.int32)
os.environ["QCHK"] = "2"
check(d, att, att, f"dense{d.n}-all")
