#!/bin/bash
# Round-2 GPU pass: parity tests, then C4 bench + phase breakdown + tie stress.
# usage: tools/gpu_r02.sh [tests|bench|all] [tag]
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
WHAT=${1:-all}; TAG=${2:-r02}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export PYTHONUNBUFFERED=1
if [ "$WHAT" = tests ] || [ "$WHAT" = all ]; then
  timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/tests.log 2>&1
  rc=$?; tail -5 $OUT/tests.log; [ $rc = 0 ] || { grep -E "FAIL|Error|error" $OUT/tests.log | head -20; exit $rc; }
fi
if [ "$WHAT" = bench ] || [ "$WHAT" = all ]; then
  for wl in ${WLS:-c4}; do
    timeout -k 10 300 python3 -u bench.py --workload $wl --steps 3 --warmup 1 --no-cpu --tie-stress "" > $OUT/bench_$wl.json 2> $OUT/bench_$wl.err || { tail -20 $OUT/bench_$wl.err; exit 1; }
    cat $OUT/bench_$wl.json
  done
  SHDPE_DEBUG=1 timeout -k 10 300 python3 -u bench.py --workload ${DEBUG_WL:-c4} --steps 1 --warmup 0 --no-cpu --tie-stress "" > $OUT/debug.json 2> $OUT/debug.err || { tail -20 $OUT/debug.err; exit 1; }
  grep shdpe $OUT/debug.err | head -20
fi
