#!/bin/bash
# A/B of engine tuning knobs on one box: bench line per setting.
# usage: tools/gpu_ab.sh TAG WORKLOAD "ENV1" "ENV2" ...   (ENV = "K=V K2=V2" or "-")
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
TAG=$1; WL=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
export PYTHONUNBUFFERED=1
i=0
for E in "$@"; do
  [ "$E" = "-" ] && E=""
  env $E SHDPE_DEBUG=${AB_DEBUG:-0} timeout -k 10 300 python3 -u bench.py --workload $WL --steps ${STEPS:-3} --warmup 1 --no-cpu --tie-stress "" > $OUT/ab$i.json 2> $OUT/ab$i.err || { tail -5 $OUT/ab$i.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open('$OUT/ab$i.json'));print('$E', '->', round(d['ms_per_step'],2),'ms', d['roofline']['kernel'], round(d['roofline']['frac'],4))"
  grep "Mcycles/batch: relax" $OUT/ab$i.err | head -2
  i=$((i+1))
done
