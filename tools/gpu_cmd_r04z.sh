# r04z: paired relax (k_batch_relax2, 16-B dist accesses): batched parity subset with SHDPE_BATCH_PAIR=1,
# then same-box A/B of C4 / C5 (pair 0 / 1 alternating, same library)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
OUT=gpurun_out/r04z; mkdir -p $OUT
QUICK='--no-cpu --tie-stress= --secondary= --host-fill 0 --d2h-rows 0 --no-stream'
line() { python3 -c "import json,sys; d=json.load(open('$1')); r=d['roofline']; print('$2', round(d['ms_per_step'],2), 'ms/step', 'kernel', round(r['avg_launch_ms'],2), 'frac', round(r['frac'],4), 'exact', round(d['ms_exact_per_step'],2), 'lanes', d.get('batch_lanes'))"; }
SHDPE_BATCH_PAIR=1 timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sizes.py tests/test_gpu_shards.py tests/test_gpu_aux.py -x -q --timeout 300 --timeout-method thread -m gpu -k "batched or multigraph or c4 or c5 or shard or tune or tie" -k "not cooperative" > $OUT/tests_pair.log 2>&1; rc=$?
tail -5 $OUT/tests_pair.log
[ $rc -ne 0 ] && { grep -n 'Error\|assert\|FAILED' $OUT/tests_pair.log | head -20; exit 1; }
for rep in 1 2; do
  for p in 0 1; do
    for wl in c4 c5; do
      SHDPE_BATCH_PAIR=$p timeout -k 10 300 python3 -u bench.py --workload $wl --steps 3 --warmup 1 $QUICK > $OUT/ab_${wl}_$p.json 2> $OUT/ab_${wl}_$p.err || { tail -20 $OUT/ab_${wl}_$p.err; exit 1; }
      line $OUT/ab_${wl}_$p.json "$wl pair=$p #$rep"
    done
  done
done
