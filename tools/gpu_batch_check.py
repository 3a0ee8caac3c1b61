"""Parity spot-check of k_batch_rows under the current SHDPE_* variant
(tools/gpu_sweep.sh runs it before timing a variant)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "shadow-1_amd"), os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402

import oracle as O  # noqa: E402
from shdpe import generators as G  # noqa: E402
from shdpe.engine import DEBUG_ENV, Engine  # noqa: E402


def check(top, att, srcs, name):
    eng = Engine(top, att, force_mode=5, debug_flags=DEBUG_ENV)
    eng.compute_rows(srcs)
    exp = O.OracleGraph(top).rows(srcs, eng.attached, threads=8)
    bad = 0
    for i, s in enumerate(srcs):
        r = eng.get_row(int(s))
        for k in ("lat", "rel", "hops", "pred", "flags"):
            a, b = r[k], exp[k][i]
            if k in ("lat", "rel"):
                a, b = a.view(np.int64), b.view(np.int64)
            if k == "flags":                 # F_EXACT (0x10) marks rows of k_exact_rows
                a, b = a & 0x0F, b & 0x0F
            if not np.array_equal(a, b):
                bad += 1
                print(f"MISMATCH {name} row {s} field {k}", flush=True)
                break
    st = eng.stats()
    eng.close()
    print(f"{name}: {len(srcs)} rows, mismatched {bad}, exact {st['rowsExact']}", flush=True)
    return bad


bad = 0
top = G.power_law(20_000, m=3, seed=4)
att = G.sample_attached(top.n, 2000, seed=2)
bad += check(top, att, att[::9], "ba20k")
top = G.random_sparse(400, 6, seed=204, quantum=1.0)
bad += check(top, np.arange(400), np.arange(400), "quantized")
top = G.random_sparse(400, 4, seed=202, directed=True)
bad += check(top, np.arange(400), np.arange(400), "directed")
top = G.random_sparse(400, 4, seed=203, vloss=True)
bad += check(top, np.arange(0, 400, 3), np.arange(0, 400, 3), "vloss")
sys.exit(1 if bad else 0)
