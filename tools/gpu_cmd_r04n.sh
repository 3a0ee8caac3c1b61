# r04n: 12-B packed arcs in the batch kernel (libshdpe_arc3.so) vs HEAD: parity subset, C4 / C5 A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
OUT=gpurun_out/r04n; mkdir -p $OUT
SHDPE_LIB=$R/shadow-1_amd/libshdpe_arc3.so timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "batched or c4 or cooperative" > $OUT/tests.log 2>&1; rc=$?; tail -3 $OUT/tests.log; [ $rc = 0 ] || { grep -E "FAIL|Error|assert" $OUT/tests.log | head -30; exit $rc; }
STAGES=ab LIBS="new arc3" WLS=c4,c5 REPS=2 bash tools/gpu_r04.sh r04n
