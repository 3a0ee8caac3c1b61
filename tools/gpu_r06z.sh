# k_direct_rows with DR_PER targets per thread at a block stride and
# non-temporal table stores: direct-path parity subset, then same-box C3a / C1
# A/B against HEAD's build (libshdpe_head)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
T=${1:-r06z}; OUT=gpurun_out/$T; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sizes.py tests/test_gpu_aux.py -x -v --timeout 300 --timeout-method thread -k "c3a or direct or shipped or complete or self or graphml" > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc = 0 ] || { grep -E "FAIL|Error|assert" $OUT/tests.log | head -20; exit $rc; }
QUICK='--no-cpu --tie-stress= --secondary= --host-fill 0 --d2h-rows 0 --no-stream'
for rep in 1 2 3; do
  for lib in new head; do
    L=$PWD/shadow-1_amd/libshdpe.so; [ $lib != new ] && L=$PWD/shadow-1_amd/libshdpe_$lib.so
    SHDPE_LIB=$L timeout -k 10 300 python3 -u bench.py --workload c3a --steps 10 --warmup 2 $QUICK > $OUT/c3a_$lib.json 2> $OUT/c3a_$lib.err || { tail -20 $OUT/c3a_$lib.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/c3a_$lib.json')); r=d['roofline']; print('c3a $lib #$rep', round(d['ms_per_step'],3), 'ms/step kernel', round(r['avg_launch_ms'],3), 'frac', round(r['frac'],4))"
  done
done
