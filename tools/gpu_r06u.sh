# AoS heap entries with the arc start + one 16-B arc record in k_exact_rows:
# exact / tie / multigraph parity subset, then same-box c4q / c5q A/B against
# HEAD's build (libshdpe_head) with the per-pop segment counters
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
T=${1:-r06u}; OUT=gpurun_out/$T; mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sizes.py tests/test_gpu_aux.py -x -v --timeout 300 --timeout-method thread -k "exact or tie or multigraph or quantized or force or c4q or c5q or c2q or self_loops or dense or path or tiefree or shipped" > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc = 0 ] || { grep -E "FAIL|Error|assert" $OUT/tests.log | head -20; exit $rc; }
QUICK='--no-cpu --tie-stress= --secondary= --host-fill 0 --d2h-rows 0 --no-stream'
for rep in 1 2; do
  for lib in new head; do
    L=$PWD/shadow-1_amd/libshdpe.so; [ $lib != new ] && L=$PWD/shadow-1_amd/libshdpe_$lib.so
    for wl in c4q c5q; do
      SHDPE_LIB=$L timeout -k 10 300 python3 -u bench.py --workload $wl --steps 2 --warmup 1 $QUICK > $OUT/${wl}_$lib.json 2> $OUT/${wl}_$lib.err || { tail -20 $OUT/${wl}_$lib.err; exit 1; }
      python3 -c "import json; d=json.load(open('$OUT/${wl}_$lib.json')); print('$wl $lib #$rep', round(d['ms_per_step'],2), 'ms/step exact', round(d['ms_exact_per_step'],2), 'ms rows_exact', d['rows_exact'])"
    done
  done
done
for lib in new head; do
  L=$PWD/shadow-1_amd/libshdpe.so; [ $lib != new ] && L=$PWD/shadow-1_amd/libshdpe_$lib.so
  SHDPE_LIB=$L SHDPE_DEBUG=1 timeout -k 10 300 python3 -u bench.py --workload c4q --steps 1 --warmup 0 $QUICK > $OUT/exactdbg_$lib.json 2> $OUT/exactdbg_$lib.err || { tail -20 $OUT/exactdbg_$lib.err; exit 1; }
  echo "== $lib"; grep -E "exact row|cyc/pop" $OUT/exactdbg_$lib.err | head -6 || true
done
