# r04zh: 4-wave variant with one vertex per group and the software pipelining (bv1_pipe4.patch) vs HEAD:
# same-box per-rank C4 shards N = 1, 4, 8, alternating
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
STAGES="shard" SHARD_NS="1 4 8" SHARD_ENVS="SHDPE_LIB=$R/shadow-1_amd/libshdpe.so;SHDPE_LIB=$R/shadow-1_amd/libshdpe_bv1pipe.so;SHDPE_LIB=$R/shadow-1_amd/libshdpe.so;SHDPE_LIB=$R/shadow-1_amd/libshdpe_bv1pipe.so" bash tools/gpu_r04.sh r04zh
