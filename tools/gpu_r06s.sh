# concurrent row sub-shards on one GPU (each its own stream / host thread, so
# one sub-shard's relax / post tail overlaps the other's work): C4 / C5 quick
# lines at K = 1 / 2 / 3 alternated, and the N=4 / N=8 shards at K = 1 / 2
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
T=${1:-r06s}; OUT=gpurun_out/$T; mkdir -p $OUT
QUICK='--no-cpu --tie-stress= --secondary= --host-fill 0 --d2h-rows 0 --no-stream'
for wl in c4 c5; do
  for rep in 1 2; do
    for K in 1 2 3; do
      [ $wl = c5 ] && [ $K = 3 ] && continue
      timeout -k 10 300 python3 -u bench.py --workload $wl --steps 3 --warmup 1 --sub-shards $K $QUICK > $OUT/${wl}_k$K.json 2> $OUT/${wl}_k$K.err || { tail -20 $OUT/${wl}_k$K.err; exit 1; }
      python3 -c "import json; d=json.load(open('$OUT/${wl}_k$K.json')); print('$wl K=$K #$rep', round(d['ms_per_step'],2), 'ms/step', round(d['value']), 'rows/s', 'exact', d['rows_exact'])"
    done
  done
done
for rep in 1 2; do
  for K in 1 2; do
    SUBK=$K timeout -k 10 300 python3 -u tools/shard_time.py c4 4 8 >> $OUT/shard.txt 2>> $OUT/shard.err || { tail -20 $OUT/shard.err; exit 1; }
  done
done
cat $OUT/shard.txt
