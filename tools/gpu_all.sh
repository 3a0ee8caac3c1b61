#!/bin/bash
# Bench line for every BASELINE config (no CPU leg) + the sparse-kernel
# phase breakdown (SHDPE_DEBUG=1) for the headline config.
# usage: tools/gpu_all.sh [workloads] [tag]
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
WLS=${1:-c1,c1m,c2,c2q,c4,c5,c3a,c3b}; TAG=${2:-all}
OUT=gpurun_out/$TAG; mkdir -p $OUT
for wl in ${WLS//,/ }; do
  echo "== $wl"
  timeout -k 10 400 python3 -u bench.py --workload $wl --steps 3 --warmup 1 --no-cpu > $OUT/bench_$wl.json 2> $OUT/bench_$wl.err || { tail -20 $OUT/bench_$wl.err; exit 1; }
  cat $OUT/bench_$wl.json
done
if [ -n "$DEBUG_WL" ]; then
  SHDPE_DEBUG=1 timeout -k 10 300 python3 -u bench.py --workload $DEBUG_WL --steps 1 --warmup 0 --no-cpu > $OUT/debug.json 2> $OUT/debug.err || { tail -20 $OUT/debug.err; exit 1; }
  cat $OUT/debug.err
fi
