#!/bin/bash
# rocprofv3 passes for one workload: kernel trace + separate PMC passes.
# usage: tools/prof_pmc.sh <workload> <outdir>
set -e
WL=${1:-c2}; OUT=${2:-gpurun_out/prof}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=/root/repo
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/trace -o trace -- python3 $R/tools/prof_run.py $WL 2
for PASS in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU" "SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"; do
  TAG=$(echo $PASS | tr ' ' '_' | cut -c1-40)
  timeout -s KILL 120 rocprofv3 --pmc $PASS --output-format csv -d $R/$OUT/pmc_$TAG -o pmc -- python3 $R/tools/prof_run.py $WL 1
done
echo PROF_DONE
