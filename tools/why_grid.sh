#!/bin/bash
# r05au: which batches of the LB 4 / 8-wave power-law case leave the fast
# path, per library build ($LIBS) and batch grid ($GRIDS; 0 = default): a
# post kernel reading another batch's distance array would fail every batch
# except those whose slot index equals their batch index
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
OUT=gpurun_out/${1:-whygrid}; mkdir -p $OUT
for lib in ${LIBS:-au pfau}; do
  for gr in ${GRIDS:-0 1 2}; do
    L=shadow-1_amd/libshdpe_$lib.so; F=$OUT/dump_${lib}_$gr.bin
    ( [ $gr != 0 ] && export SHDPE_BATCH_GRID=$gr; SHDPE_LIB=$R/$L SHDPE_DEBUG=1 SHDPE_DUMP_BATCHES=$F SHDPE_BATCH_LB=4 SHDPE_BATCH_WPE=8 \
      timeout -k 10 120 python3 -u tools/lb8_probe.py rows > $OUT/grid_${lib}_$gr.txt 2> $OUT/grid_${lib}_$gr.err ) || { echo "$lib grid $gr failed"; tail -5 $OUT/grid_${lib}_$gr.err; exit 1; }
    python3 - $F "$lib grid $gr" <<'PY'
import sys, numpy as np
raw = np.fromfile(sys.argv[1], dtype=np.int32)
nB, LB = int(raw[0]), int(raw[1])
dbg = raw[2 + nB * LB: 2 + nB * LB + 16 * nB].reshape(nB, 16)
bad = np.nonzero(dbg[:, 3])[0]
print(sys.argv[2], "batches", nB, "tie batches", len(bad), "ok batches", sorted(set(range(nB)) - set(bad.tolist()))[:12])
PY
  done
done
