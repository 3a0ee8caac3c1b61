#!/bin/bash
# batched-kernel parity tests + c4 timing with phase stats
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out/batch
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "batched" --timeout 120 --timeout-method thread > gpurun_out/batch/tests.log 2>&1 || { tail -40 gpurun_out/batch/tests.log; exit 1; }
tail -3 gpurun_out/batch/tests.log
for wl in ${1:-c4}; do
SHDPE_DEBUG=1 timeout -k 10 300 python3 -u bench.py --workload $wl --steps 1 --warmup 0 --no-cpu > gpurun_out/batch/$wl.json 2> gpurun_out/batch/$wl.err || { tail -20 gpurun_out/batch/$wl.err; exit 1; }
cat gpurun_out/batch/$wl.json gpurun_out/batch/$wl.err
done
