#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out/ws
for G in 256 64 16; do
  echo "== grid $G"
  SHDPE_BATCH_GRID=$G SHDPE_BATCH_DELTA_FACTOR=1000 SHDPE_DEBUG=1 QROWS=${QROWS:-4096} timeout -k 10 200 python3 -u tools/gpu_configs_quick.py c4 2> gpurun_out/ws/g$G.err || { tail gpurun_out/ws/g$G.err; exit 1; }
  grep "shdpe" gpurun_out/ws/g$G.err | tail -3
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 --list-avail > $R/gpurun_out/ws/avail.txt 2>&1 || true
