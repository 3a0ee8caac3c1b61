#!/bin/bash
# rocprofv3 kernel trace + stats of one bench step: tools/prof_kernels.sh <workload> <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; WL=${1:-c3b}; TAG=${2:-prof}; OUT=$R/gpurun_out/$TAG
mkdir -p $OUT; cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 $R/bench.py --workload $WL --steps 1 --warmup 0 --no-cpu > $OUT/bench.json 2> $OUT/err.log || { tail -5 $OUT/err.log; exit 1; }
cut -d, -f1-4 $OUT/trace/trace_kernel_stats.csv | cut -c1-160
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print('$WL ms/step', d['ms_per_step'], 'frac', d['roofline']['frac'])"
