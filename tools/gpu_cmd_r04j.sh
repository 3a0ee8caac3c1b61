# r04j: cooperative relax on LB-8 batches for small shards: parity, then per-rank shard times at N=4, 8
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
OUT=gpurun_out/r04j; mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "cooperative" > $OUT/tests.log 2>&1; rc=$?; tail -3 $OUT/tests.log; [ $rc = 0 ] || { grep -E "FAIL|Error|assert" $OUT/tests.log | head -30; exit $rc; }
STAGES=shard SHARD_NS="4 8" SHARD_ENVS="X=0;SHDPE_BATCH_COOP=2 SHDPE_BATCH_LB=8;SHDPE_BATCH_COOP=4 SHDPE_BATCH_LB=8;SHDPE_BATCH_COOP=2 SHDPE_BATCH_LB=8 SHDPE_BATCH_POST_SUB=1;SHDPE_BATCH_COOP=2 SHDPE_BATCH_LB=8 SHDPE_BATCH_WPE=8" bash tools/gpu_r04.sh r04j
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "c5" > $OUT/tests_c5.log 2>&1; rc=$?; tail -3 $OUT/tests_c5.log; [ $rc = 0 ] || exit $rc
STAGES=bench WLS=c5 bash tools/gpu_r04.sh r04j
