# r04l: HEAD after the shared-device guard: shard / batched / coop GPU tests, the one-GPU rehearsal of
# the self-launched 2-rank bench, driver-default bench, rocprof trace + PMC traffic of C4 (new source hash)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
PYTEST_K="shard or batched or cooperative or tune or c4" STAGES="tests rehearse default trace pmc" WLS=c4 bash tools/gpu_r04.sh r04l
