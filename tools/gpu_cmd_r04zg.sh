# r04zg: final HEAD checks: full GPU suite, rocprof traces of C5 / C3a / C2, 2-rank rehearsal
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
STAGES="tests" bash tools/gpu_r04.sh r04zg || exit 1
STAGES="trace" WLS=c5,c3a,c2 bash tools/gpu_r04.sh r04zg || exit 1
STAGES="rehearse" bash tools/gpu_r04.sh r04zg
