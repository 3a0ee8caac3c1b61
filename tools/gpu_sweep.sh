#!/bin/bash
# Sweep SHDPE_* variants on one workload (debug counters on): one bench step
# each.  usage: VARIANTS="SHDPE_BATCH_DELTA_FACTOR=2 ..." tools/gpu_sweep.sh c4 tag
# (a variant is a comma-joined list of VAR=VALUE)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
WL=${1:-c4}; TAG=${2:-sweep}; OUT=gpurun_out/$TAG; mkdir -p $OUT
for v in $VARIANTS; do
  echo "== $v"
  if [ -n "$CHECK" ]; then env ${v//,/ } timeout -k 10 200 python3 -u tools/gpu_batch_check.py > $OUT/$v.check 2>&1 || { cat $OUT/$v.check | tail; exit 1; }; tail -1 $OUT/$v.check; fi
  env ${v//,/ } SHDPE_DEBUG=${DBG:-1} timeout -k 10 200 python3 -u bench.py --workload $WL --steps ${STEPS:-1} --warmup ${WARM:-0} --no-cpu --tie-stress "" --d2h-rows 0 --no-stream > $OUT/$v.json 2> $OUT/$v.err || { tail -20 $OUT/$v.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('ms/step %.1f' % d['ms_per_step'], 'kernel %.1f' % d['roofline']['avg_launch_ms'], 'exact', d['rows_exact'])" $OUT/$v.json
  grep -E "Mcycles/batch: relax|vertex-procs|arc-visits" $OUT/$v.err
done
