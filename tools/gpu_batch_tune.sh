#!/bin/bash
# batched kernel tuning: timing only, over "LB:deltaFactor" pairs
# usage: tools/gpu_batch_tune.sh <workload> "<LB:DF ...>" [tag]
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
WL=${1:-c4}; TAG=${3:-tune}; OUT=gpurun_out/$TAG; mkdir -p $OUT
for cfg in ${2:-"16:2"}; do
  LB=${cfg%%:*}; DF=${cfg##*:}; F=$OUT/${WL}_lb${LB}_df${DF}
  SHDPE_BATCH_LB=$LB SHDPE_BATCH_DELTA_FACTOR=$DF timeout -k 10 300 python3 -u bench.py --workload $WL --steps 2 --warmup 1 --no-cpu > $F.json 2> $F.err || { tail -20 $F.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('$WL LB=$LB DF=$DF ms/step', round(d['ms_per_step'],1), 'frac', round(d['roofline']['frac'],4), 'exact', d['rows_exact'])" $F.json
done
