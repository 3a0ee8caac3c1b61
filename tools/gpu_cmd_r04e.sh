# r04e: multigraph support -- the new multigraph parity tests + aux helpers + the batched / tie subsets
mkdir -p gpurun_out/r04e
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "multigraph or aux or is_complete or tie or golden or shim" > gpurun_out/r04e/tests.log 2>&1; rc=$?; tail -5 gpurun_out/r04e/tests.log; [ $rc = 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/r04e/tests.log | head -30; exit $rc; }
