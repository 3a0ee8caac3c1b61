# r04r: load-batch widths around the new default (relax BK / post BKP = 3 / 3): 2 / 2, 3 / 2, 2 / 3
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
STAGES=ab LIBS="new bk2 bk3p2 bk2p3" WLS=c4,c5 REPS=2 bash tools/gpu_r04.sh r04r
