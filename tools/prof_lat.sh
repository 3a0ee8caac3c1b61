#!/bin/bash
set -e
WL=${1:-c2}; OUT=${2:-gpurun_out/prof_lat}
mkdir -p $OUT; cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=/root/repo
for PASS in "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_sum" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_ATOMIC_WITH_RET_REQ_sum TCP_TCC_ATOMIC_WITHOUT_RET_REQ_sum TCP_PENDING_STALL_CYCLES_sum" "SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CU_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SMEM"; do
  TAG=$(echo $PASS | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --pmc $PASS --output-format csv -d $R/$OUT/$TAG -o pmc -- python3 $R/tools/prof_run.py $WL 1
done
echo PROF_DONE
