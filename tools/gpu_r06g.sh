# cooperative relax on the GPU: its parity tests (each variant, abort path),
# the C4 eight-shard full-size table with it forced and with the tune's pick,
# then per-rank shard times N=1 / 8 plain vs forced vs tuned (same box)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
T=${1:-r06g}; mkdir -p gpurun_out/$T
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "cooperative" > gpurun_out/$T/coop_tests.log 2>&1
rc=$?; tail -3 gpurun_out/$T/coop_tests.log; [ $rc = 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/$T/coop_tests.log | head -20; exit $rc; }
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_shards.py -x -v --timeout 300 --timeout-method thread -k "eight_shards" > gpurun_out/$T/shards.log 2>&1
rc=$?; tail -3 gpurun_out/$T/shards.log; [ $rc = 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/$T/shards.log | head -20; exit $rc; }
SHARD_NS="1 8" SHARD_ENVS="X=0;SHDPE_BATCH_COOP=-1;SHDPE_BATCH_COOP=2;SHDPE_BATCH_COOP=2 SHDPE_BATCH_COOP_WPE=6;SHDPE_BATCH_COOP=2 SHDPE_BATCH_COOP_WPE=4;X=1" SHARD_WL=c4 STAGES=shard tools/gpu_r05.sh $T
# r05au: the rejected label-walk prefetch (pf) and diagnostic builds on the
# LB 4 / 8-wave power-law case: why each batch leaves the fast path
LIBS="new diag pfdiag pf" tools/why_probe.sh $T
grep -h "\[diag\] viol" gpurun_out/$T/why_*.err | head -30
