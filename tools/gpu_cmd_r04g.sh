# r04g: exact kernel with the next pop's record + first arcs prefetched (libshdpe_pfonly.so): parity subset, A/B vs HEAD
mkdir -p gpurun_out/r04g
SHDPE_LIB=$PWD/shadow-1_amd/libshdpe_pfonly.so timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "exact or tie or quantized or quantised or golden or c4q or c5q or multigraph or shipped or path" > gpurun_out/r04g/tests.log 2>&1; rc=$?; tail -4 gpurun_out/r04g/tests.log; [ $rc = 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/r04g/tests.log | head -30; exit $rc; }
STAGES=ab LIBS="exbase pfonly" WLS=c4q,c5q REPS=2 bash tools/gpu_r04.sh r04g
