# r04m: k_direct_rows with 4 targets per thread and vector non-temporal stores: parity, A/B on C3a vs HEAD
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
OUT=gpurun_out/r04m; mkdir -p $OUT
true
STAGES=ab LIBS="drbase new dr4plain dr1nt" WLS=c3a REPS=2 bash tools/gpu_r04.sh r04m
