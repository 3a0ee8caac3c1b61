"""Time k_exact_rows per row on a few graphs (forced exact mode)."""
import os, sys, time
sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "shadow-1_amd")]
import numpy as np
from shdpe import generators as G
from shdpe.engine import Engine

cases = [("rgg2000", G.rgg(2000, seed=1), None), ("rgg10k", G.rgg(10_000, seed=1), None),
         ("rgg10k_T64", G.rgg(10_000, seed=1), 64)]
for name, top, nt in cases:
    att = np.arange(top.n, dtype=np.int32) if nt is None else G.sample_attached(top.n, nt, seed=1)
    for per_cu in (None,):
        eng = Engine(top, att, force_mode=3)
        eng.compute_rows(att[:1])
        eng.reset_stats()
        srcs = att[1:5]
        eng.compute_rows(srcs)
        st = eng.stats()
        print(name, "ms/row", st["msExactKernel"] / len(srcs), "rows", st["rowsExact"], flush=True)
        eng.close()
