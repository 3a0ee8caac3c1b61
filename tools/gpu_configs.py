"""Parity (sampled rows vs oracle) + timing for the larger BASELINE configs."""
import os, sys, time
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(R, "shadow-1_amd"), os.path.join(R, "oracle")]
import numpy as np
from shdpe import generators as G
from shdpe.engine import Engine, DEBUG_ENV
from oracle import OracleGraph

for wl in sys.argv[1].split(","):
    t0 = time.time(); top, att = G.make_config(wl); tg = time.time() - t0
    eng = Engine(top, att, debug_flags=DEBUG_ENV if any(k.startswith('SHDPE_') for k in os.environ) else 0)
    st0 = eng.stats()
    nrows = int(os.environ.get("QROWS", "2048"))
    nrows = min(nrows, eng.T)
    eng.compute_positions(0, min(256, nrows)); eng.reset_stats()
    t0 = time.time(); eng.compute_positions(0, nrows); dt = time.time() - t0
    st = eng.stats()
    print(f"{wl}: n={st['nVertices']} arcs={st['nArcs']} T={eng.T} gen={tg:.1f}s rows={nrows} "
          f"kernel_ms={st['msSparseKernel']:.1f} exact_rows={st['rowsExact']} exact_ms={st['msExactKernel']:.1f} "
          f"rows/s={nrows/(st['msTotal']/1e3):.0f} -> full table est {eng.T/(nrows/(st['msTotal']/1e3)):.2f}s", flush=True)
    og = OracleGraph(top)
    rng = np.random.default_rng(0)
    srcs = eng.attached[rng.choice(nrows, int(os.environ.get('PROWS', '6')), replace=False)]
    bad = 0
    t0 = time.time()
    exp = og.rows(srcs, eng.attached, threads=8)
    to = time.time() - t0
    for i, s in enumerate(srcs):
        g = eng.get_row(int(s))
        ok = all(np.array_equal(g[k].view(np.int64) if k in ('lat','rel') else g[k], exp[k][i].view(np.int64) if k in ('lat','rel') else exp[k][i]) for k in ('lat','rel','hops','pred'))
        bad += not ok
    print(f"{wl}: parity sampled rows={len(srcs)} bad={bad} (oracle {to/len(srcs)*8:.2f}s/row/thread)", flush=True)
    eng.close()
