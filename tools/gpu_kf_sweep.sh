#!/bin/bash
# Sparse-kernel variant sweep (SHDPE_KFLAGS) on one workload: timing line +
# SHDPE_DEBUG phase breakdown per variant.
# usage: tools/gpu_kf_sweep.sh <workload> "<kflags list>" [tag]
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
WL=${1:-c2}; KFS=${2:-0}; TAG=${3:-kf}
OUT=gpurun_out/$TAG; mkdir -p $OUT
for kf in $KFS; do
  SHDPE_KFLAGS=$kf timeout -k 10 120 python3 -u bench.py --workload $WL --steps 3 --warmup 1 --no-cpu > $OUT/${WL}_$kf.json 2> $OUT/${WL}_$kf.err || { tail -20 $OUT/${WL}_$kf.err; exit 1; }
  SHDPE_KFLAGS=$kf SHDPE_DEBUG=1 timeout -k 10 120 python3 -u bench.py --workload $WL --steps 1 --warmup 0 --no-cpu > /dev/null 2> $OUT/${WL}_${kf}_dbg.err || { tail -20 $OUT/${WL}_${kf}_dbg.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/${WL}_$kf.json')); print('kf=$kf', round(d['ms_per_step'],2), 'ms', round(d['roofline']['frac'],4))"
  grep shdpe $OUT/${WL}_${kf}_dbg.err | cut -c1-400
done
