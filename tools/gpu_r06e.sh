# cooperative relax: parity (small cases, the C4 8-shard table), abort path,
# N=8 shard times plain vs forced vs tuned; r05au diag probe
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out/r06e
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "cooperative" > gpurun_out/r06e/coop_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r06e/coop_tests.log; [ $rc = 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/r06e/coop_tests.log | head -20; exit $rc; }
SHARD_NS="8" SHARD_ENVS="X=0;SHDPE_BATCH_COOP=2;SHDPE_BATCH_COOP=2 SHDPE_BATCH_COOP_WPE=6;SHDPE_TUNE_LOG=1" STAGES=shard tools/gpu_r05.sh r06e || exit 1
grep "tune" gpurun_out/r06e/shard.err | tail -8
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_shards.py -x -v --timeout 300 --timeout-method thread -k "eight_shards" > gpurun_out/r06e/shards.log 2>&1
rc=$?; tail -3 gpurun_out/r06e/shards.log; [ $rc = 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/r06e/shards.log | head -20; exit $rc; }
LIBS="pfaudiag" tools/why_probe.sh r06e
