#!/bin/bash
# Round-5 GPU pass.  Stages (space-separated in $STAGES):
#   tests     pytest -m gpu (PYTEST_K filters)
#   rehearse  BENCH_REHEARSE_ONE_GPU=1 bench.py --gpus 2: the self-launched
#             N-rank flow on one GPU; asserts "n_gpus": 2 and a verified
#             table assembly (allgather.verified, host transport)
#   shard     per-rank shard times (tools/shard_time.py) for $SHARD_WL at
#             N = $SHARD_NS, once per SHDPE_* setting in $SHARD_ENVS (';' list)
#   envs      quick bench lines for $WLS per SHDPE_* setting in $ENVS (';' list)
#   bench     quick bench.py lines for $WLS (no CPU leg / extras)
#   default   the driver's command (python bench.py, all legs)
#   trace     rocprofv3 --kernel-trace --stats of quick bench lines for $WLS
#   pmc       FETCH_SIZE / WRITE_SIZE / TCC hit+miss passes -> traffic_<wl>.json
#   hostfill  bench's host_fill block alone (C4)
#   exactdbg  k_exact_rows per-pop cycle counters on c4q (SHDPE_DEBUG)
#   exactpmc  k_exact_rows SQ instruction counters on c4q
# usage: STAGES="tests bench" tools/gpu_r05.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
TAG=${1:-r05}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export PYTHONUNBUFFERED=1
WLS=${WLS:-c4}
QUICK='--no-cpu --tie-stress= --secondary= --host-fill 0 --d2h-rows 0 --no-stream'
line() { python3 -c "import json,sys; d=json.load(open('$1')); r=d['roofline']; print('$2', round(d['value']), 'rows/s', round(d['ms_per_step'],2), 'ms/step', 'kernel', round(r['avg_launch_ms'],2), 'ms frac', round(r['frac'],4), 'exact', round(d['ms_exact_per_step'],2), 'lanes', d.get('batch_lanes'))"; }
for st in ${STAGES:-tests bench}; do
  case $st in
  tests)
    timeout -k 10 1100 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/tests.log 2>&1
    rc=$?; tail -3 $OUT/tests.log; [ $rc = 0 ] || { grep -E "FAIL|Error|error|assert" $OUT/tests.log | head -30; exit $rc; } ;;
  rehearse)
    BENCH_REHEARSE_ONE_GPU=1 timeout -k 10 300 python3 -u bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu --tie-stress "" --secondary "" --host-fill 0 --no-stream > $OUT/rehearse.json 2> $OUT/rehearse.err || { tail -20 $OUT/rehearse.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/rehearse.json')); a=d.get('allgather', {}); assert d['n_gpus']==2 and a.get('verified'), d; print('rehearse n_gpus', d['n_gpus'], round(d['value']), 'rows/s', round(d['ms_per_step'],2), 'ms/step; allgather', a.get('transport'), round(a['ms']), 'ms verified', a['verified'])" || exit 1 ;;
  shard)
    IFS=';' read -ra ES <<< "${SHARD_ENVS:-X=0}"
    for e in "${ES[@]}"; do
      env $e timeout -k 10 400 python3 -u tools/shard_time.py ${SHARD_WL:-c4} ${SHARD_NS:-1 2 4 8} >> $OUT/shard.txt 2>> $OUT/shard.err || { tail -20 $OUT/shard.err; exit 1; }
    done
    cat $OUT/shard.txt ;;
  sharddbg)
    # k_batch_rows counters (per-batch cost spread, phases, arc visits) of
    # rank 0's shard at N = $SHARD_NS
    SHDPE_DEBUG=1 timeout -k 10 400 python3 -u tools/shard_time.py ${SHARD_WL:-c4} ${SHARD_NS:-8} > $OUT/sharddbg.txt 2> $OUT/sharddbg.err || { tail -20 $OUT/sharddbg.err; exit 1; }
    cat $OUT/sharddbg.txt; grep "shdpe\] .*batch" $OUT/sharddbg.err | tail -12 ;;
  ab)
    # same-box A/B of library builds (tools/build_variant.sh): LIBS="new x y"
    # -> shadow-1_amd/libshdpe_<x>.so (new = the in-tree libshdpe.so), REPS
    # rounds alternating, quick C4 lines
    for wl in ${WLS//,/ }; do
      for rep in $(seq 1 ${REPS:-2}); do
        for lib in ${LIBS:-new}; do
          L=shadow-1_amd/libshdpe.so; [ $lib != new ] && L=shadow-1_amd/libshdpe_$lib.so
          SHDPE_LIB=$R/$L timeout -k 10 300 python3 -u bench.py --workload $wl --steps 3 --warmup 1 $QUICK > $OUT/ab_${wl}_$lib.json 2> $OUT/ab_${wl}_$lib.err || { tail -20 $OUT/ab_${wl}_$lib.err; exit 1; }
          line $OUT/ab_${wl}_$lib.json "$wl $lib #$rep"
        done
      done
    done ;;
  envs)
    # quick bench lines for $WLS once per SHDPE_* setting in $ENVS (';' list), REPS rounds
    IFS=';' read -ra ES <<< "${ENVS:-X=0}"
    for wl in ${WLS//,/ }; do
      for rep in $(seq 1 ${REPS:-1}); do
        for e in "${ES[@]}"; do
          T2=$(echo "$e" | tr ' =/' '_-_' | cut -c1-60)
          env $e timeout -k 10 300 python3 -u bench.py --workload $wl --steps ${STEPS:-3} --warmup 1 $QUICK > $OUT/env_${wl}_$T2.json 2> $OUT/env_${wl}_$T2.err || { tail -20 $OUT/env_${wl}_$T2.err; exit 1; }
          line $OUT/env_${wl}_$T2.json "$wl [$e] #$rep"
        done
      done
    done ;;
  bench)
    for wl in ${WLS//,/ }; do
      timeout -k 10 300 python3 -u bench.py --workload $wl --steps ${STEPS:-3} --warmup 1 $QUICK > $OUT/bench_$wl.json 2> $OUT/bench_$wl.err || { tail -20 $OUT/bench_$wl.err; exit 1; }
      line $OUT/bench_$wl.json $wl
    done ;;
  default)
    timeout -k 10 600 python3 -u bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -20 $OUT/bench_default.err; exit 1; }
    line $OUT/bench_default.json "default" ;;
  trace)
    for wl in ${WLS//,/ }; do
      (cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/trace_$wl -o trace -- python3 $R/bench.py --workload $wl --steps 5 --warmup 1 $QUICK > $R/$OUT/trace_$wl.json 2> $R/$OUT/trace_$wl.err) || { tail -20 $OUT/trace_$wl.err; exit 1; }
      line $OUT/trace_$wl.json "$wl traced"
    done ;;
  pmc)
    for wl in ${WLS//,/ }; do
      for PASS in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_ATOMIC_sum TCC_ATOMIC_sum" ${EXTRA_PASSES}; do
        T2=$(echo $PASS | tr ' ' '_' | cut -c1-40)
        (cd /tmp && TMPDIR=/tmp timeout -s KILL 150 rocprofv3 --pmc $PASS --output-format csv -d $R/$OUT/pmc_${wl}_$T2 -o pmc -- python3 $R/bench.py --workload $wl --steps 1 --warmup 0 $QUICK > $R/$OUT/pmc_${wl}_$T2.log 2>&1) || { echo "pmc pass $wl $PASS failed"; tail -5 $OUT/pmc_${wl}_$T2.log; exit 1; }
      done
      python3 tools/traffic_json.py $OUT $wl $TAG $OUT/traffic_$wl.json $OUT/${TAG}_${wl}_pmc || exit 1
    done ;;
  hostfill)
    # the host_fill block alone (C4: rows path + fresh-engine fill_rowstore)
    SHDPE_FILL_LOG=1 timeout -k 10 400 python3 -u bench.py --workload c4 --steps 3 --warmup 1 --no-cpu --tie-stress= --secondary= --d2h-rows 0 --no-stream > $OUT/hostfill.json 2> $OUT/hostfill.err || { tail -20 $OUT/hostfill.err; exit 1; }
    python3 -c "import json; h=json.load(open('$OUT/hostfill.json'))['host_fill']; print({k: (round(v, 3) if isinstance(v, float) else v) for k, v in h.items() if k not in ('how', 'rows_path')}); print('rows_path', {k: (round(v, 3) if isinstance(v, float) else v) for k, v in h['rows_path'].items() if k != 'how'})"
    grep "fill_rowstore" $OUT/hostfill.err || true ;;
  exactdbg)
    # k_exact_rows per-pop segment counters (SHDPE_DEBUG) on the c4q tie rows
    SHDPE_DEBUG=1 timeout -k 10 300 python3 -u bench.py --workload c4q --steps 1 --warmup 0 $QUICK > $OUT/exactdbg.json 2> $OUT/exactdbg.err || { tail -20 $OUT/exactdbg.err; exit 1; }
    grep "exact row" $OUT/exactdbg.err | sort -t= -k2 -n -r | head -20 || true ;;
  exactpmc)
    # instruction mix of the exact kernel (SQ counters, one pass)
    (cd /tmp && TMPDIR=/tmp timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY --output-format csv -d $R/$OUT/exactpmc -o pmc -- python3 $R/bench.py --workload c4q --steps 1 --warmup 0 $QUICK > $R/$OUT/exactpmc.log 2>&1) || { echo "exact pmc failed"; tail -5 $OUT/exactpmc.log; exit 1; }
    find $OUT/exactpmc -name "*counter_collection.csv" | head -1 | xargs grep -h "k_exact_rows" | head -20 || true ;;
  esac
done
