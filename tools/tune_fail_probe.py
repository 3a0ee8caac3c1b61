"""shd_pe_tune with one variant failing every batch (SHDPE_TUNE_FAIL_WPE):
the tune log (per candidate: times, exact rows, exclusion) and the pick."""
import os, sys
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(R, "shadow-1_amd")]
from shdpe import generators as G
from shdpe.engine import Engine, DEBUG_ENV
top = G.power_law(8000, m=3, seed=14)
att = G.sample_attached(top.n, 1200, seed=3)
eng = Engine(top, att, force_mode=5, debug_flags=DEBUG_ENV)
eng.tune()
st = eng.stats()
print({k: st[k] for k in ("batchLanes", "batchWaves", "batchPostWaves", "rowsExact", "rowsComputed")}, flush=True)
eng.compute_all()
st = eng.stats()
print({k: st[k] for k in ("batchLanes", "batchWaves", "batchPostWaves", "rowsExact", "rowsComputed")}, flush=True)
eng.close()
