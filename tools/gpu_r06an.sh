# dense early-stop tie rows in one launch with a dynamic row take (up to 4096
# dense tie slots): dense parity subset, then same-box c3bq A/B against HEAD
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
T=${1:-r06an}; OUT=gpurun_out/$T; mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sizes.py -x -v --timeout 400 --timeout-method thread -k "dense or c3b" > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc = 0 ] || { grep -E "FAIL|Error|assert" $OUT/tests.log | head -20; exit $rc; }
QUICK='--no-cpu --tie-stress= --secondary= --host-fill 0 --d2h-rows 0 --no-stream'
for rep in 1 2; do
  for lib in new head; do
    L=$PWD/shadow-1_amd/libshdpe.so; [ $lib != new ] && L=$PWD/shadow-1_amd/libshdpe_$lib.so
    SHDPE_LIB=$L timeout -k 10 300 python3 -u bench.py --workload c3bq --steps 2 --warmup 1 $QUICK > $OUT/c3bq_$lib.json 2> $OUT/c3bq_$lib.err || { tail -20 $OUT/c3bq_$lib.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/c3bq_$lib.json')); print('c3bq $lib #$rep', round(d['ms_per_step'],1), 'ms/step exact', round(d['ms_exact_per_step'],1), 'rows_exact', d['rows_exact'])"
  done
done
