# r04f: exact kernel with LDS tail windows + speculative next-pop record: parity subset, then A/B vs HEAD on c4q / c5q
mkdir -p gpurun_out/r04f
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "exact or tie or quantized or quantised or golden or c4q or c5q or multigraph or shipped or path" > gpurun_out/r04f/tests.log 2>&1; rc=$?; tail -4 gpurun_out/r04f/tests.log; [ $rc = 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/r04f/tests.log | head -30; exit $rc; }
STAGES=ab LIBS="exbase new" WLS=c4q,c5q REPS=2 bash tools/gpu_r04.sh r04f
