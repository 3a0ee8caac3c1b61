# sub-shards continued: C5 at K = 2 with the 6-wave relax forced (the tune of
# a lone sub-shard picked 4 waves), C4 K = 2 with 6-wave relax, N = 2 shard at
# K = 1 / 2
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
T=${1:-r06t}; OUT=gpurun_out/$T; mkdir -p $OUT
QUICK='--no-cpu --tie-stress= --secondary= --host-fill 0 --d2h-rows 0 --no-stream'
run() {  # tag workload K [env...]
  local tag=$1 wl=$2 K=$3; shift 3
  env "$@" timeout -k 10 300 python3 -u bench.py --workload $wl --steps 3 --warmup 1 --sub-shards $K $QUICK > $OUT/$tag.json 2> $OUT/$tag.err || { tail -20 $OUT/$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$tag.json')); print('$tag', round(d['ms_per_step'],2), 'ms/step', 'waves', d.get('batch_kernel_waves'), d.get('batch_post_kernel_waves'), 'exact', d['rows_exact'])"
}
for rep in 1 2; do


  run c4_k1_r$rep c4 1 X=0
  run c4_k2_r$rep c4 2 X=0
  run c4_k2w6_r$rep c4 2 SHDPE_BATCH_WPE=6
done
for rep in 1 2; do
  for K in 1 2; do
    SUBK=$K timeout -k 10 300 python3 -u tools/shard_time.py c4 2 >> $OUT/shard.txt 2>> $OUT/shard.err || { tail -20 $OUT/shard.err; exit 1; }
  done
done
cat $OUT/shard.txt
