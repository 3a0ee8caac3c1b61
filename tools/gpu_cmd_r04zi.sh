# r04zi: load-batch widths on the pipelined kernel (relax BK 2 / 4, predecessor BKP 2) vs HEAD (3 / 3),
# same box, alternating, quick C4 / C5 lines
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
STAGES="ab" WLS=c4,c5 LIBS="new bk2 bk4 bkp2" REPS=2 bash tools/gpu_r04.sh r04zi
