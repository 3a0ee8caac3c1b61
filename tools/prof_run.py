"""Run one workload's full table once (for rocprofv3 passes)."""
import os, sys
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(R, "shadow-1_amd")]
from shdpe import generators as G
from shdpe.engine import Engine
wl = sys.argv[1] if len(sys.argv) > 1 else "c2"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
top, att = G.make_config(wl)
eng = Engine(top, att)
for _ in range(reps):
    eng.compute_all()
st = eng.stats()
print(wl, "rows", st["rowsComputed"], "sparse_ms", round(st["msSparseKernel"], 2), "launches", st["launchesSparse"], flush=True)
eng.close()
