"""Timing only (no parity) of the first QROWS rows of a config."""
import os, sys, time
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(R, "shadow-1_amd")]
from shdpe import generators as G
from shdpe.engine import Engine
wl = sys.argv[1]
top, att = G.make_config(wl)
eng = Engine(top, att)
nrows = min(int(os.environ.get("QROWS", "4096")), eng.T)
eng.compute_positions(0, nrows)
st = eng.stats()
print(f"{wl}: rows={nrows} kernel_ms={st['msSparseKernel']:.1f} total_ms={st['msTotal']:.1f} "
      f"rows/s={nrows / (st['msTotal'] / 1e3):.0f}", flush=True)
eng.close()
