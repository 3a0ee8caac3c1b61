# deferred tie export (k_tie_export after the post kernel instead of a full
# predecessor pass in line): batched / tie / shard parity subset, then
# same-box A/B against HEAD's build (libshdpe_head): C4, C5, c4q, c5q
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
T=${1:-r06af}; OUT=gpurun_out/$T; mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sizes.py tests/test_gpu_shards.py -x -v --timeout 300 --timeout-method thread -k "batched or tie or c4 or c5 or tune or cooperative or multigraph or quantized or exact or shard or deep or vertex_loss" > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc = 0 ] || { grep -E "FAIL|Error|assert" $OUT/tests.log | head -20; exit $rc; }
QUICK='--no-cpu --tie-stress= --secondary= --host-fill 0 --d2h-rows 0 --no-stream'
for rep in 1 2; do
  for lib in new head; do
    L=$PWD/shadow-1_amd/libshdpe.so; [ $lib != new ] && L=$PWD/shadow-1_amd/libshdpe_$lib.so
    for wl in c4 c4q c5 c5q; do
      SHDPE_LIB=$L timeout -k 10 300 python3 -u bench.py --workload $wl --steps 3 --warmup 1 $QUICK > $OUT/${wl}_$lib.json 2> $OUT/${wl}_$lib.err || { tail -20 $OUT/${wl}_$lib.err; exit 1; }
      python3 -c "import json; d=json.load(open('$OUT/${wl}_$lib.json')); print('$wl $lib #$rep', round(d['ms_per_step'],2), 'ms/step main', round(d['roofline']['avg_launch_ms'],2), 'exact', round(d['ms_exact_per_step'],2), 'rows_exact', d['rows_exact'])"
    done
  done
done
