# r04i: C5 in one round of dist arrays (libshdpe_d160.so: budget 96 -> 160 GiB) vs HEAD; C4 post kernel over half batches
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
OUT=gpurun_out/r04i; mkdir -p $OUT
STAGES=ab LIBS="new d160" WLS=c5 REPS=2 bash tools/gpu_r04.sh r04i || exit 1
QUICK='--no-cpu --tie-stress= --secondary= --host-fill 0 --d2h-rows 0 --no-stream'
for rep in 1 2; do
for e in "X=0" "SHDPE_BATCH_POST_SUB=1"; do
  env $e timeout -k 10 200 python3 -u bench.py --workload c4 --steps 3 --warmup 1 $QUICK > $OUT/c4_$e.json 2> $OUT/c4_$e.err || { tail -5 $OUT/c4_$e.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/c4_$e.json')); print('c4 $e #$rep', round(d['ms_per_step'],2), 'ms', round(d['roofline']['frac'],4), d['batch_kernel_waves'], d['batch_post_kernel_waves'])"
done
done
