# r04ze: same-box per-rank C4 shard times, pipelined HEAD vs the r04v relax (libshdpe_unpipe.so), alternating
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
STAGES="shard" SHARD_NS="1 4 8" SHARD_ENVS="SHDPE_LIB=$R/shadow-1_amd/libshdpe.so;SHDPE_LIB=$R/shadow-1_amd/libshdpe_unpipe.so;SHDPE_LIB=$R/shadow-1_amd/libshdpe.so;SHDPE_LIB=$R/shadow-1_amd/libshdpe_unpipe.so" bash tools/gpu_r04.sh r04ze
