# r04zd: HEAD profile set after the software pipelining (part 2): rocprof traces of C5 / C3a / C2,
# per-rank C4 shard times at N = 1, 2, 4, 8, 2-rank rehearsal
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
STAGES="trace" WLS=c5,c3a,c2 bash tools/gpu_r04.sh r04zd || exit 1
STAGES="shard rehearse" WLS=c4 SHARD_NS="1 2 4 8" bash tools/gpu_r04.sh r04zd
