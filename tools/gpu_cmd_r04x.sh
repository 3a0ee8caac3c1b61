# r04x: C4 environment sweep on the r04v kernel (delta factor, heavy degree, LB 32), base runs interleaved
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
OUT=gpurun_out/r04x; mkdir -p $OUT
QUICK='--no-cpu --tie-stress= --secondary= --host-fill 0 --d2h-rows 0 --no-stream'
line() { python3 -c "import json,sys; d=json.load(open('$1')); r=d['roofline']; print('$2', round(d['ms_per_step'],2), 'ms/step', 'kernel', round(r['avg_launch_ms'],2), 'frac', round(r['frac'],4), 'lanes', d.get('batch_lanes'))"; }
i=0
for cfg in base SHDPE_BATCH_DELTA_FACTOR=0.6 SHDPE_BATCH_DELTA_FACTOR=1.0 base SHDPE_HEAVY_DEG=32 SHDPE_HEAVY_DEG=128 SHDPE_BATCH_LB=32 base SHDPE_BATCH_DELTA_FACTOR=0.6 SHDPE_BATCH_DELTA_FACTOR=1.0; do
  i=$((i+1)); E=""; [ $cfg != base ] && E=$cfg
  env $E timeout -k 10 300 python3 -u bench.py --workload c4 --steps 3 --warmup 1 $QUICK > $OUT/s$i.json 2> $OUT/s$i.err || { tail -20 $OUT/s$i.err; exit 1; }
  line $OUT/s$i.json "c4 $cfg"
done
