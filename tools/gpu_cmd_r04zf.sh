# r04zf: pipelining gated to the 8 / 6-wave variants: batched parity subset, same-box per-rank shard
# A/B against the r04v relax (libshdpe_unpipe.so), then the HEAD profile set (default bench, trace, PMC)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
OUT=gpurun_out/r04zf; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sizes.py tests/test_gpu_shards.py -x -q --timeout 300 --timeout-method thread -m gpu -k "batched or c4_whole or c4q or c5 or each_lb or multigraph or shard or tune" -k "not cooperative" > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log
[ $rc -ne 0 ] && { grep -n 'Error\|assert\|FAILED' $OUT/tests.log | head -20; exit 1; }
STAGES="shard" SHARD_NS="1 4 8" SHARD_ENVS="SHDPE_LIB=$R/shadow-1_amd/libshdpe.so;SHDPE_LIB=$R/shadow-1_amd/libshdpe_unpipe.so;SHDPE_LIB=$R/shadow-1_amd/libshdpe.so;SHDPE_LIB=$R/shadow-1_amd/libshdpe_unpipe.so" bash tools/gpu_r04.sh r04zf || exit 1
STAGES="default trace pmc" WLS=c4 bash tools/gpu_r04.sh r04zf
