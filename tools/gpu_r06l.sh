# dense predecessor pass by chunk minima (SHDPE_PRED_CM=1): dense parity tests
# with it, then C3b alternating with the per-k-step pass; C4 with SGPR
# spills to scratch (libshdpe_nosv) against the in-tree build, same box
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
T=${1:-r06l}; mkdir -p gpurun_out/$T
SHDPE_PRED_CM=1 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sizes.py -x -v --timeout 200 --timeout-method thread -k "dense or c3b" > gpurun_out/$T/dense_cm.log 2>&1
rc=$?; echo "dense tests CM rc=$rc"; tail -2 gpurun_out/$T/dense_cm.log; [ $rc = 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/$T/dense_cm.log | head -20; exit $rc; }
WLS=c3b ENVS="SHDPE_PRED_CM=0;SHDPE_PRED_CM=1;SHDPE_PRED_CM=0;SHDPE_PRED_CM=1;SHDPE_PRED_CM=1 SHDPE_PRED_MI=3" STEPS=1 STAGES=envs tools/gpu_r05.sh $T || exit 1
LIBS="new nosv" REPS=2 WLS=c4 STAGES=ab tools/gpu_r05.sh $T
