# r04k: HEAD final profile set: full GPU suite (small batched shards now relax cooperatively), per-rank
# shard times at N = 1, 2, 4, 8, driver-default bench, rocprof trace + PMC traffic of C4
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
STAGES="tests shard default trace pmc" WLS=c4 SHARD_NS="1 2 4 8" bash tools/gpu_r04.sh r04k
