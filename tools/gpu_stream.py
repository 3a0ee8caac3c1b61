"""Probe shd_pe_stream_bandwidth at a few workgroups-per-CU settings."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
code = ("import sys; sys.path.insert(0, %r); from shdpe import generators as G; "
        "from shdpe.engine import Engine; import numpy as np; top = G.random_sparse(100, 4, seed=1); "
        "e = Engine(top, np.arange(100)); print(round(e.stream_bandwidth(), 1)); e.close()"
        % os.path.join(ROOT, "shadow-1_amd"))
for wg in sys.argv[1:] or ["4", "8", "16", "32"]:
    env = dict(os.environ, SHDPE_STREAM_WG_PER_CU=wg)
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                         timeout=120)
    print("wg/CU", wg, out.stdout.strip(), out.stderr.strip()[-200:])
