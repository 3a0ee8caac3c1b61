# hub-cell count of the batch source order (SHDPE_BATCH_HUBS): C4 quick lines
# and the N=8 shard per setting
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
T=${1:-r06ac}; OUT=gpurun_out/$T; mkdir -p $OUT
ENVS="X=0;SHDPE_BATCH_HUBS=64;SHDPE_BATCH_HUBS=128;SHDPE_BATCH_HUBS=512;SHDPE_BATCH_HUBS=1024;SHDPE_BATCH_HUBS=2048" REPS=2 WLS=c4 STAGES=envs tools/gpu_r05.sh $T || exit 1
SHARD_NS="8" SHARD_ENVS="X=0;SHDPE_BATCH_HUBS=64;SHDPE_BATCH_HUBS=512;SHDPE_BATCH_HUBS=1024;SHDPE_BATCH_HUBS=2048;X=0" SHARD_WL=c4 STAGES=shard tools/gpu_r05.sh $T
