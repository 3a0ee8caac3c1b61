# r04c: predecessor records (libshdpe_rec.so) vs HEAD (libshdpe.so): A/B + full GPU parity of rec
export STAGES="ab" LIBS="new rec" WLS=c4,c4q,c5 REPS=2
bash tools/gpu_r04.sh r04c || exit 1
SHDPE_LIB=$PWD/shadow-1_amd/libshdpe_rec.so timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04c/tests_rec.log 2>&1; rc=$?; tail -3 gpurun_out/r04c/tests_rec.log; [ $rc = 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/r04c/tests_rec.log | head -20; exit $rc; }
