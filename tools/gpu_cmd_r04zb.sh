# r04zb: software-pipelined light-vertex loop (pipe1) + predecessor pass (new) (next take's dist / row range in flight during the
# current take's arcs): quick parity, then same-box A/B against the r04v relax (libshdpe_base.so)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
OUT=gpurun_out/r04zb; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sizes.py -x -q --timeout 300 --timeout-method thread -m gpu -k "batched or c4_whole or c4q or c5 or each_lb or multigraph_rows" -k "not cooperative" > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log
[ $rc -ne 0 ] && { grep -n 'Error\|assert\|FAILED' $OUT/tests.log | head -20; exit 1; }
STAGES="ab" WLS=c4,c5 LIBS="new pipe1 pipe2 base" REPS=2 bash tools/gpu_r04.sh r04zb
