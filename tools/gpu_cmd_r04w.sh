# r04w: same-box A/B of the 12-B packed arc layout in the batch kernel (tools/variants/arc3_batch.patch)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
STAGES="ab" WLS=c4,c5 LIBS="new arc3" REPS=2 bash tools/gpu_r04.sh r04w
