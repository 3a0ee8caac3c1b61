# r04t: 32-bit label-walk step counter (the walk loop of the post kernel loses its spills) and the
# cooperative relax's group state pinned to scalar registers (coop relax spills 39 -> 28 at 8 waves)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
OUT=gpurun_out/r04t; mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "batched or cooperative or c4 or tie or deep or path" > $OUT/tests.log 2>&1; rc=$?; tail -3 $OUT/tests.log; [ $rc = 0 ] || { grep -E "FAIL|Error|assert" $OUT/tests.log | head -30; exit $rc; }
STAGES=ab LIBS="headt new" WLS=c4,c5 REPS=2 bash tools/gpu_r04.sh r04t || exit 1
STAGES=shard SHARD_NS="4 8" bash tools/gpu_r04.sh r04t
