# r04p: batch-kernel debug counters / timestamps moved from registers to LDS (relax spills 56 -> 26 at
# 8 waves, 10 -> 0 at 4): batched parity, C4 / C5 A/B vs HEAD, a debug-counter run, shard times
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
OUT=gpurun_out/r04p; mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "batched or cooperative or c4 or tune or shard or tie" > $OUT/tests.log 2>&1; rc=$?; tail -3 $OUT/tests.log; [ $rc = 0 ] || { grep -E "FAIL|Error|assert" $OUT/tests.log | head -30; exit $rc; }
STAGES=ab LIBS="headk2 new" WLS=c4,c5 REPS=2 bash tools/gpu_r04.sh r04p || exit 1
STAGES="shard sharddbg" SHARD_NS="1 2 4 8" bash tools/gpu_r04.sh r04p
