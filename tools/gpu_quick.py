"""Quick GPU parity + timing probe (dev tool)."""
import os, sys, time
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(R, "shadow-1_amd"), os.path.join(R, "oracle")]
import numpy as np
from shdpe import generators as G
from shdpe.engine import Engine
from oracle import OracleGraph

def cmp(top, att, force=0, tag=""):
    og = OracleGraph(top)
    eng = Engine(top, att, force_mode=force)
    t0 = time.time(); eng.compute_all(); dt = time.time() - t0
    bad = 0
    for i, s in enumerate(eng.attached):
        g = eng.get_row(int(s)); o = og.row(int(s), eng.attached)
        ok = (np.array_equal(g['lat'].view(np.int64), o['lat'].view(np.int64)) and
              np.array_equal(g['rel'].view(np.int64), o['rel'].view(np.int64)) and
              np.array_equal(g['hops'], o['hops']) and np.array_equal(g['pred'], o['pred']))
        if not ok:
            bad += 1
            if bad <= 2:
                k = np.flatnonzero((g['lat'] != o['lat']) | (g['rel'] != o['rel']) | (g['hops'] != o['hops']) | (g['pred'] != o['pred']))
                print(tag, "row", s, "first bad cols", k[:5], g['lat'][k[:3]], o['lat'][k[:3]], g['hops'][k[:3]], o['hops'][k[:3]], g['pred'][k[:3]], o['pred'][k[:3]], g['flags'][k[:3]], o['flags'][k[:3]])
    st = eng.stats()
    print(f"{tag}: rows={len(eng.attached)} bad_rows={bad} exact_rows={st['rowsExact']} t={dt:.3f}s sparse_ms={st['msSparseKernel']:.2f} exact_ms={st['msExactKernel']:.2f}", flush=True)
    eng.close()
    return bad

tot = 0
for seed in range(3):
    tot += cmp(G.random_sparse(200, 5, seed), np.arange(200), tag=f"rand{seed}")
tot += cmp(G.random_sparse(300, 4, 7, directed=True), np.arange(300), tag="directed")
tot += cmp(G.random_sparse(300, 4, 8, vloss=True), np.arange(0, 300, 2), tag="vloss")
tot += cmp(G.random_sparse(300, 6, 9, quantum=1.0), np.arange(300), tag="quantized")
tot += cmp(G.random_sparse(300, 6, 9, quantum=1.0), np.arange(300), force=3, tag="forced-exact")
print("TOTAL BAD", tot, flush=True)
top, att = G.make_config("c2")
os.environ["SHDPE_DEBUG"] = os.environ.get("QDEBUG", "1")
for kf in os.environ.get("QKFLAGS", "0").split(","):
  os.environ["SHDPE_KFLAGS"] = kf
  for lay in os.environ.get("QLAYOUTS", "2,3").split(","):
    os.environ["SHDPE_LAYOUT"] = lay
    eng = Engine(top, att); eng.compute_positions(0, 512); eng.reset_stats()
    eng.compute_all(); st = eng.stats()
    print(f"C2 kflags={kf} layout={lay}: sparse_ms={st['msSparseKernel']:.2f} rows/s={10000/(st['msTotal']/1e3):.0f}", flush=True)
    eng.close()
