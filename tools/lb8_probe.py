"""LB-8 / 4-wave batch probe (tools only): the test_batched_kernel_each_lb
power-law case with SHDPE_DEBUG counters, for comparing library builds."""
import os, sys
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(R, "shadow-1_amd")]
from shdpe import generators as G
from shdpe.engine import Engine, DEBUG_ENV
top = G.power_law(8000, m=3, seed=15)
att = G.sample_attached(top.n, 1203, seed=4)
eng = Engine(top, att, force_mode=5, debug_flags=DEBUG_ENV)
mode = sys.argv[1] if len(sys.argv) > 1 else "all"
if mode == "all":
    eng.compute_positions(0, eng.T)
else:                                   # the test's sources: every third attached vertex
    eng.compute_rows(att[::3])
st = eng.stats()
print({k: st[k] for k in ("batchLanes", "batchWaves", "batchPostWaves", "rowsExact", "rowsTieEarly", "rowsComputed")})
eng.close()
