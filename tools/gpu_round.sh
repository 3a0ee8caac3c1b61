#!/bin/bash
# Verify HEAD on the GPU: parity tests, then bench lines for the given
# workloads (no CPU leg), then optional env-variant probes on C2.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
TAG=${1:-chk}; WLS=${2:-c2,c4}; OUT=gpurun_out/$TAG; mkdir -p $OUT
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
  tail -3 $OUT/gpu_tests.log
fi
for wl in ${WLS//,/ }; do
  timeout -k 10 300 python3 -u bench.py --workload $wl --steps 3 --warmup 1 --no-cpu > $OUT/bench_$wl.json 2> $OUT/bench_$wl.err || { tail -20 $OUT/bench_$wl.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/bench_$wl.json')); print('$wl', round(d['value']), round(d['ms_per_step'],2), 'ms', round(d['roofline']['frac'],4))"
done
for v in $PROBES; do   # e.g. PROBES="SHDPE_BATCH=1:c2 SHDPE_BATCH=1,SHDPE_BATCH_LB=32:c2"
  envs=${v%%:*}; wl=${v##*:}
  env ${envs//,/ } timeout -k 10 300 python3 -u bench.py --workload $wl --steps 3 --warmup 1 --no-cpu > $OUT/probe.json 2> $OUT/probe.err || { echo "probe $v failed"; tail -20 $OUT/probe.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/probe.json')); print('$v', round(d['value']), round(d['ms_per_step'],2), 'ms')"
done
