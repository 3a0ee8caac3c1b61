# r04s: uniform LDS-derived values pinned to scalar registers (relax spills 21 -> 17 at 8 waves, 6 -> 2 at 6)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
OUT=gpurun_out/r04s; mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "batched or cooperative or c4 or tie" > $OUT/tests.log 2>&1; rc=$?; tail -3 $OUT/tests.log; [ $rc = 0 ] || { grep -E "FAIL|Error|assert" $OUT/tests.log | head -30; exit $rc; }
STAGES=ab LIBS="headq new" WLS=c4,c5 REPS=2 bash tools/gpu_r04.sh r04s || exit 1
STAGES=shard SHARD_NS="1 2 4 8" bash tools/gpu_r04.sh r04s
