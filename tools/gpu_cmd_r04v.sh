# r04v: HEAD final profile set: full GPU suite, per-rank shard times at N = 1, 2, 4, 8, driver-default
# bench, rocprof trace + PMC traffic of C4, rocprof trace of C5 / C3a / C2, 2-rank rehearsal
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
STAGES="tests shard default trace pmc rehearse" WLS=c4 SHARD_NS="1 2 4 8" bash tools/gpu_r04.sh r04v || exit 1
STAGES="trace" WLS=c5,c3a,c2 bash tools/gpu_r04.sh r04v
