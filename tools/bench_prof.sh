#!/bin/bash
# Round profile capture for the bench workload: bench line, rocprofv3 kernel
# trace + stats of the same command, and separate PMC passes for HBM bytes.
set -e
WL=${1:-c2}; TAG=${2:-r01}; OUT=gpurun_out/bench_$TAG
mkdir -p $OUT
R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=/root/repo
cd $R
timeout -k 10 300 python3 -u bench.py --workload $WL --steps 5 --warmup 2 > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/trace -o trace -- python3 $R/bench.py --workload $WL --steps 5 --warmup 2 --no-cpu --tie-stress "" > $R/$OUT/bench_traced.json
for PASS in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
  T2=$(echo $PASS | cut -d' ' -f1)
  timeout -s KILL 150 rocprofv3 --pmc $PASS --output-format csv -d $R/$OUT/pmc_$T2 -o pmc -- python3 $R/bench.py --workload $WL --steps 1 --warmup 0 --no-cpu --tie-stress "" > /dev/null
done
echo BENCH_PROF_DONE
