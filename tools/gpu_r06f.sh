# r05au: first phase-2 violation per batch of the failing variant; cooperative
# relax shapes at the C4 N=8 shard (LB 16 and K = 4 combinations)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out/r06f
LIBS="pfdx" tools/why_probe.sh r06f || exit 1
grep "viol batch" gpurun_out/r06f/why_pfdx.err | head -12
SHARD_NS="8" SHARD_ENVS="SHDPE_BATCH_LB=16;SHDPE_BATCH_LB=16 SHDPE_BATCH_COOP=2 SHDPE_BATCH_COOP_WPE=4;SHDPE_BATCH_COOP=2 SHDPE_BATCH_COOP_WPE=4;SHDPE_BATCH_LB=16 SHDPE_BATCH_COOP=4 SHDPE_BATCH_COOP_WPE=8;SHDPE_BATCH_LB=16 SHDPE_BATCH_COOP=4 SHDPE_BATCH_COOP_WPE=6;SHDPE_BATCH_COOP=4 SHDPE_BATCH_COOP_WPE=6;SHDPE_BATCH_COOP=3 SHDPE_BATCH_COOP_WPE=6" STAGES=shard tools/gpu_r05.sh r06f
