# hub-cell count vs shard size (SHDPE_BATCH_HUBS): N=8 / 4 / 2 shards
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
T=${1:-r06ad}; OUT=gpurun_out/$T; mkdir -p $OUT
for rep in 1 2; do
  SHARD_NS="8" SHARD_ENVS="X=0;SHDPE_BATCH_HUBS=32;SHDPE_BATCH_HUBS=48;SHDPE_BATCH_HUBS=64;SHDPE_BATCH_HUBS=96" SHARD_WL=c4 STAGES=shard tools/gpu_r05.sh $T > /dev/null || exit 1
  SHARD_NS="4" SHARD_ENVS="X=0;SHDPE_BATCH_HUBS=32;SHDPE_BATCH_HUBS=64;SHDPE_BATCH_HUBS=128" SHARD_WL=c4 STAGES=shard tools/gpu_r05.sh $T > /dev/null || exit 1
  SHARD_NS="2" SHARD_ENVS="X=0;SHDPE_BATCH_HUBS=64;SHDPE_BATCH_HUBS=128" SHARD_WL=c4 STAGES=shard tools/gpu_r05.sh $T > /dev/null || exit 1
done
cat $OUT/shard.txt
