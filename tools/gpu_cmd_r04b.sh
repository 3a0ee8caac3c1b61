export STAGES="ab" LIBS="base new fetch" WLS=c4 REPS=2
bash tools/gpu_r04.sh r04b || exit 1
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "batched or tune or c4" > gpurun_out/r04b/tests_new.log 2>&1; rc=$?; tail -3 gpurun_out/r04b/tests_new.log; [ $rc = 0 ] || exit $rc
SHDPE_LIB=$PWD/shadow-1_amd/libshdpe_fetch.so timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "batched or tune or c4" > gpurun_out/r04b/tests_fetch.log 2>&1; rc=$?; tail -3 gpurun_out/r04b/tests_fetch.log; [ $rc = 0 ] || exit $rc
STAGES=shard SHARD_ENVS="X=0;SHDPE_BATCH_COOP=2;SHDPE_BATCH_COOP=4;SHDPE_BATCH_COOP=2 SHDPE_BATCH_POST_SUB=1" bash tools/gpu_r04.sh r04b
