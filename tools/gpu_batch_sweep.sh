#!/bin/bash
# batched kernel: timing/phase stats over LB and delta factor for one workload
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out/sweep
WL=${1:-c4}
for cfg in ${2:-"16:2 8:2 8:1 8:4"}; do
  LB=${cfg%%:*}; DF=${cfg##*:}
  echo "== $WL LB=$LB dF=$DF"
  SHDPE_BATCH=1 SHDPE_BATCH_LB=$LB SHDPE_BATCH_DELTA_FACTOR=$DF SHDPE_DEBUG=1 timeout -k 10 300 python3 -u bench.py --workload $WL --steps 1 --warmup 0 --no-cpu > gpurun_out/sweep/${WL}_$LB_$DF.json 2> gpurun_out/sweep/${WL}_$LB_$DF.err || { tail -20 gpurun_out/sweep/${WL}_$LB_$DF.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('ms/step', round(d['ms_per_step'],1), 'rows/s', round(d['value']), 'frac', round(d['roofline']['frac'],4), 'exact', d['rows_exact'])" gpurun_out/sweep/${WL}_$LB_$DF.json
  grep shdpe gpurun_out/sweep/${WL}_$LB_$DF.err
done
