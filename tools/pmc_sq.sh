#!/bin/bash
# SQ issue / wait breakdown and TA busy per kernel of one quick bench line:
# tools/pmc_sq.sh <tag> <workload>   (one rocprofv3 --pmc pass per counter set)
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; OUT=gpurun_out/$1; WL=${2:-c2}; mkdir -p $OUT
Q="--workload $WL --steps 1 --warmup 0 --no-cpu --tie-stress= --secondary= --host-fill 0 --d2h-rows 0 --no-stream"
i=0
for P in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" "SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT" "TA_BUSY_avr TA_BUSY_max"; do
  i=$((i+1))
  (cd /tmp && TMPDIR=/tmp timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $R/$OUT/${WL}_p$i -o pmc -- python3 $R/bench.py $Q > $R/$OUT/${WL}_p$i.log 2>&1) || { echo "pass $i failed"; tail -5 $OUT/${WL}_p$i.log; exit 1; }
  find $OUT/${WL}_p$i -name "*counter_collection.csv" | head -1 | xargs python3 -c "
import csv,sys,collections
s=collections.defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    k=r['Kernel_Name'].split('(')[0][-40:]
    s[(k,r['Counter_Name'])]+=float(r['Counter_Value'])
for (k,c),v in sorted(s.items()): print('$i', k, c, '%.4g'%v)
"
done
