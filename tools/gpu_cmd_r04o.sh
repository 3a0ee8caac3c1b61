# r04o: cooperative relax as its own instantiation (PART 3) with agent-scope dist loads: coop / batched
# parity (tie-free runs must send no row to the exact kernel), C4 N=1 A/B vs HEAD, shard times N=4, 8
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
OUT=gpurun_out/r04o; mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "cooperative or batched or tie_relevance or shard" > $OUT/tests.log 2>&1; rc=$?; tail -3 $OUT/tests.log; [ $rc = 0 ] || { grep -E "FAIL|Error|assert" $OUT/tests.log | head -30; exit $rc; }
STAGES=ab LIBS="headk new" WLS=c4 REPS=2 bash tools/gpu_r04.sh r04o || exit 1
STAGES=shard SHARD_NS="4 8" bash tools/gpu_r04.sh r04o
