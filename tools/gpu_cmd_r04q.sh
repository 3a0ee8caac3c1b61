# r04q: load-batch widths: relax BK 4 / post BKP 3 (bkp3), BK 3 / BKP 3 (bk3) vs HEAD (4 / 4)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
STAGES=ab LIBS="new bkp3 bk3" WLS=c4,c5 REPS=2 bash tools/gpu_r04.sh r04q
