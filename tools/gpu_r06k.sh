# new GPU tests first (tune guard against a failing variant, one-rank RCCL
# gather), then the whole GPU suite and the smoke entry point
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
T=${1:-r06k}; mkdir -p gpurun_out/$T
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "tune_never or one_rank" > gpurun_out/$T/new_tests.log 2>&1
rc=$?; tail -3 gpurun_out/$T/new_tests.log; [ $rc = 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/$T/new_tests.log | head -20; exit $rc; }
STAGES=tests tools/gpu_r05.sh $T || exit 1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1; rc=$?; tail -2 gpurun_out/$T/smoke.log; exit $rc
