# r05au on the round-5 tree (6ce98cf): plain (audiag) vs the label-walk
# prefetch patch (pfau, pfaudiag), LB 4 / 8 waves, violations printed; then
# the dense predecessor pass with the packed-argument register budget:
# parity of every dense test at MI 4 and 6, C3b per MI against HEAD's pass
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
T=${1:-r06h}; mkdir -p gpurun_out/$T
LIBS="audiag pfaudiag pfau" tools/why_probe.sh $T
grep -h "\[diag\]" gpurun_out/$T/why_*.err | head -40
for mi in 4 6; do
  SHDPE_PRED_MI=$mi timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sizes.py -x -v --timeout 200 --timeout-method thread -k "dense or c3b" > gpurun_out/$T/dense_mi$mi.log 2>&1
  rc=$?; echo "dense tests MI=$mi rc=$rc"; tail -2 gpurun_out/$T/dense_mi$mi.log; [ $rc = 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/$T/dense_mi$mi.log | head -20; exit $rc; }
done
WLS=c3b ENVS="SHDPE_PRED_MI=2;SHDPE_PRED_MI=3;SHDPE_PRED_MI=4;SHDPE_PRED_MI=6;SHDPE_LIB=$PWD/shadow-1_amd/libshdpe_head.so" STEPS=1 STAGES=envs tools/gpu_r05.sh $T
# the label-walk prefetch at HEAD (it passes the LB 4 / 8-wave case there):
# same-box C4 / C5 A/B against the in-tree build
LIBS="new pf" REPS=2 WLS=c4 STAGES=ab tools/gpu_r05.sh $T
# cooperative relax shapes on LB-16 batches at the N=8 shard
SHARD_NS="8" SHARD_ENVS="SHDPE_BATCH_LB=16;SHDPE_BATCH_LB=16 SHDPE_BATCH_COOP=2 SHDPE_BATCH_COOP_WPE=4;SHDPE_BATCH_LB=16 SHDPE_BATCH_COOP=2 SHDPE_BATCH_COOP_WPE=8;SHDPE_BATCH_COOP=4 SHDPE_BATCH_COOP_WPE=8" SHARD_WL=c4 STAGES=shard tools/gpu_r05.sh ${T}s
