# r04zc: HEAD profile set after the software pipelining (part 1): full GPU suite, driver-default
# bench, rocprof trace + PMC traffic of C4
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
STAGES="tests default trace pmc" WLS=c4 bash tools/gpu_r04.sh r04zc
