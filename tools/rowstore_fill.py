"""Host fill rate of the dense row store (CPU only): a whole T x T table of
synthetic engine rows through shd_rowstore_store_row (one row at a time) and
shd_rowstore_store_rows (blocks, threaded).  C4 size by default (T = 16,384,
n = 100k).  python tools/rowstore_fill.py [T] [block] [threads]"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "shadow-1_amd"))
from shdpe.engine import RowStore  # noqa: E402

T = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
B = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
TH = int(sys.argv[3]) if len(sys.argv) > 3 else 0
n = max(100_000, T)
rng = np.random.default_rng(0)
att = np.sort(rng.choice(n, size=T, replace=False)).astype(np.int32)
lat = rng.uniform(1, 500, size=(B, T))
rel = rng.uniform(0.5, 1, size=(B, T))
flags = np.zeros((B, T), np.uint8)
out = {"T": T, "block": B}
st = RowStore(n, att)
k = min(T, 512)
t0 = time.perf_counter()
for i in range(k):
    st.store_row(int(att[i]), lat[i % B], rel[i % B], flags[i % B])
out["store_row_rows_per_s"] = k / (time.perf_counter() - t0)
st.close()
st = RowStore(n, att)
t0 = time.perf_counter()
for b0 in range(0, T, B):
    c = min(B, T - b0)
    st.store_rows(att[b0:b0 + c], lat[:c], rel[:c], flags[:c], threads=TH)
dt = time.perf_counter() - t0
out.update(store_rows_s=dt, store_rows_rows_per_s=T / dt, entries=int(st.size()),
           memory_GB=st.memory_bytes() / 1e9, threads=TH or "default")
print(json.dumps(out))
