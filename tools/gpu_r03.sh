#!/bin/bash
# Round-3 GPU pass.  Stages (space-separated in $STAGES):
#   tests   pytest -m gpu (PYTEST_K filters)
#   bench   bench.py lines for $WLS (no CPU leg, no tie stress)
#   ab      same-box A/B: libshdpe_head.so vs libshdpe.so on $WLS, twice each
#   debug   SHDPE_DEBUG counters of k_batch_rows on $DEBUG_WL
#   relabel tools/relabel_probe.py
# usage: STAGES="tests bench" tools/gpu_r03.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
TAG=${1:-r03}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export PYTHONUNBUFFERED=1
WLS=${WLS:-c4}
line() { python3 -c "import json,sys; d=json.load(open('$1')); r=d['roofline']; print('$2', round(d['value']), 'rows/s', round(d['ms_per_step'],2), 'ms/step', 'kernel', round(r['avg_launch_ms'],2), 'ms frac', round(r['frac'],4), 'exact', round(d['ms_exact_per_step'],2))"; }
for st in ${STAGES:-tests bench}; do
  case $st in
  tests)
    timeout -k 10 1100 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/tests.log 2>&1
    rc=$?; tail -3 $OUT/tests.log; [ $rc = 0 ] || { grep -E "FAIL|Error|error|assert" $OUT/tests.log | head -30; exit $rc; } ;;
  bench)
    for wl in ${WLS//,/ }; do
      timeout -k 10 300 python3 -u bench.py --workload $wl --steps ${STEPS:-3} --warmup 1 --no-cpu --tie-stress "" --d2h-rows 0 --no-stream > $OUT/bench_$wl.json 2> $OUT/bench_$wl.err || { tail -20 $OUT/bench_$wl.err; exit 1; }
      line $OUT/bench_$wl.json $wl
    done ;;
  ab)
    # same-box A/B of library builds: LIBS="head new x" -> shadow-1_amd/libshdpe_<x>.so
    # (new = libshdpe.so); REPS rounds, alternating
    for wl in ${WLS//,/ }; do
      for rep in $(seq 1 ${REPS:-2}); do
        for lib in ${LIBS:-head new}; do
          L=shadow-1_amd/libshdpe.so; [ $lib != new ] && L=shadow-1_amd/libshdpe_$lib.so
          SHDPE_LIB=$R/$L timeout -k 10 300 python3 -u bench.py --workload $wl --steps 3 --warmup 1 --no-cpu --tie-stress "" --d2h-rows 0 --no-stream > $OUT/ab_${wl}_$lib.json 2> $OUT/ab_${wl}_$lib.err || { tail -20 $OUT/ab_${wl}_$lib.err; exit 1; }
          line $OUT/ab_${wl}_$lib.json "$wl $lib #$rep"
          if [ -n "$ABDEBUG" ]; then SHDPE_LIB=$R/$L SHDPE_DEBUG=1 timeout -k 10 300 python3 -u bench.py --workload $wl --steps 1 --warmup 0 --no-cpu --tie-stress "" --d2h-rows 0 --no-stream > /dev/null 2> $OUT/abdbg_${wl}_$lib.err || exit 1; grep shdpe $OUT/abdbg_${wl}_$lib.err | head -8; fi
        done
      done
    done ;;
  debug)
    SHDPE_DEBUG=1 timeout -k 10 300 python3 -u bench.py --workload ${DEBUG_WL:-c4} --steps 1 --warmup 0 --no-cpu --tie-stress "" --d2h-rows 0 --no-stream > $OUT/debug.json 2> $OUT/debug.err || { tail -20 $OUT/debug.err; exit 1; }
    grep shdpe $OUT/debug.err | head -20 ;;
  pmc)
    # L2-miss traffic of one launch per workload: FETCH_SIZE / WRITE_SIZE /
    # TCC hit+miss in separate passes (MI355X_MICROARCH.md HBM section)
    for wl in ${WLS//,/ }; do
      for PASS in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" ${EXTRA_PASSES}; do
        T2=$(echo $PASS | tr ' ' '_' | cut -c1-40)
        (cd /tmp && TMPDIR=/tmp timeout -s KILL 150 rocprofv3 --pmc $PASS --output-format csv -d $R/$OUT/pmc_${wl}_$T2 -o pmc -- python3 $R/bench.py --workload $wl --steps 1 --warmup 0 --no-cpu --tie-stress "" --d2h-rows 0 --no-stream > $R/$OUT/pmc_${wl}_$T2.log 2>&1) || { echo "pmc pass $wl $PASS failed"; tail -5 $OUT/pmc_${wl}_$T2.log; exit 1; }
      done
      python3 tools/traffic_json.py $OUT $wl $TAG $OUT/traffic_$wl.json || exit 1
    done ;;
  trace)
    for wl in ${WLS//,/ }; do
      (cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/trace_$wl -o trace -- python3 $R/bench.py --workload $wl --steps 5 --warmup 1 --no-cpu --tie-stress "" --d2h-rows 0 --no-stream > $R/$OUT/trace_$wl.json 2> $R/$OUT/trace_$wl.err) || { tail -20 $OUT/trace_$wl.err; exit 1; }
      line $OUT/trace_$wl.json "$wl traced"
    done ;;
  default)
    # the driver's command: python bench.py (defaults: C4, CPU legs, tie stress, D2H)
    timeout -k 10 600 python3 -u bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -20 $OUT/bench_default.err; exit 1; }
    line $OUT/bench_default.json "default" ;;
  envsweep)
    # one line per environment setting in $ENVS (';'-separated lists of VAR=VAL)
    IFS=';' read -ra ES <<< "${ENVS:-}"
    for e in "${ES[@]}"; do
      for wl in ${WLS//,/ }; do
        env $e SHDPE_DEBUG=${ABDEBUG:-0} timeout -k 10 300 python3 -u bench.py --workload $wl --steps 3 --warmup 1 --no-cpu --tie-stress "" --d2h-rows 0 --no-stream > $OUT/env.json 2> $OUT/env.err || { tail -20 $OUT/env.err; exit 1; }
        line $OUT/env.json "$wl [$e]"
        if [ -n "$ABDEBUG" ]; then grep shdpe $OUT/env.err | head -8; fi
      done
    done ;;
  relabel)
    timeout -k 10 400 python3 -u tools/relabel_probe.py ${RELABEL_WL:-c4} > $OUT/relabel.txt 2>&1 || { tail -20 $OUT/relabel.txt; exit 1; }
    cat $OUT/relabel.txt ;;
  esac
done
