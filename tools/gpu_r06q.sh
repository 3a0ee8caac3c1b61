# flattened per-lane label walks in the post kernel: batched parity subset +
# the full C4 table, then same-box C4 / C5 A/B against HEAD's build
# (libshdpe_head) and the N=8 shard
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
T=${1:-r06r}; mkdir -p gpurun_out/$T
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sizes.py -x -v --timeout 300 --timeout-method thread -k "batched_kernel_each or c4_whole_table or c4q or c5 or tie_slot or tune or cooperative or deep or vertex_loss or multigraph" > gpurun_out/$T/tests.log 2>&1
rc=$?; tail -2 gpurun_out/$T/tests.log; [ $rc = 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/$T/tests.log | head -20; exit $rc; }
LIBS="new head" REPS=2 WLS=c4,c5 STAGES=ab tools/gpu_r05.sh $T || exit 1
SHARD_NS="8" SHARD_ENVS="X=0;SHDPE_LIB=$PWD/shadow-1_amd/libshdpe_head.so;X=0;SHDPE_LIB=$PWD/shadow-1_amd/libshdpe_head.so" SHARD_WL=c4 STAGES=shard tools/gpu_r05.sh $T
