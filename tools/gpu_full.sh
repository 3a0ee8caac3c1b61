#!/bin/bash
# Full GPU pass at HEAD: parity tests, default bench line (C4 + CPU baseline
# + tie stress), rocprofv3 kernel stats of the C4 bench.
# usage: tools/gpu_full.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
TAG=${1:-full}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export PYTHONUNBUFFERED=1
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
  rc=$?; tail -3 $OUT/tests.log; [ $rc = 0 ] || { grep -E "FAIL|Error" $OUT/tests.log | head -20; exit $rc; }
fi
timeout -k 10 600 python3 -u bench.py ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o trace -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu --tie-stress "" --d2h-rows 0 ${PROF_ARGS} > $R/$OUT/prof_bench.json 2> $R/$OUT/prof.err || { tail -20 $R/$OUT/prof.err; exit 1; }
find $R/$OUT/prof -name "*kernel_stats.csv" | head -1 | xargs head -12
