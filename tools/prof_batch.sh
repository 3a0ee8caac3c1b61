#!/bin/bash
# PMC passes (one per counter set) over a short run of the batched kernel.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; OUT=$R/gpurun_out/pmc_${TAG:-b}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
export SHDPE_BATCH_DELTA_FACTOR=${DF:-1000} QROWS=${QROWS:-4096}
i=0
for PASS in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_VALU" "FETCH_SIZE TCC_HIT_sum" "SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_WAVES SQ_BUSY_CYCLES SQ_INST_CYCLES_VMEM_RD SQ_INSTS_FLAT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $PASS --output-format csv -d $OUT/p$i -o pmc -- python3 $R/tools/gpu_configs_quick.py ${WL:-c4} > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 $R/tools/summarize_pmc.py $OUT
