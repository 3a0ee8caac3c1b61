#!/bin/bash
# One bench line per BASELINE config (GPU only, no CPU leg) -> gpurun_out/<tag>/configs.jsonl
# usage: tools/gpu_configs_bench.sh <tag> [workloads]
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
TAG=${1:-cfg}; WLS=${2:-"c1 c1m c2 c2q c3a c3b c4 c4q c5"}
OUT=gpurun_out/$TAG; mkdir -p $OUT; : > $OUT/configs.jsonl
export PYTHONUNBUFFERED=1
for wl in $WLS; do
  steps=3; [ $wl = c3b ] && steps=2; [ $wl = c5 ] && steps=2
  timeout -k 10 400 python3 -u bench.py --workload $wl --steps $steps --warmup 1 --no-cpu --tie-stress "" --d2h-rows 0 --no-stream > $OUT/b_$wl.json 2> $OUT/b_$wl.err || { echo "FAIL $wl"; tail -5 $OUT/b_$wl.err; exit 1; }
  tail -1 $OUT/b_$wl.json >> $OUT/configs.jsonl
  python3 -c "import json,sys; d=json.loads(open('$OUT/b_$wl.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$wl', round(d['ms_per_step'],2), int(d['value']), r['kernel'], round(r['frac'],4), d['rows_exact'])"
done
