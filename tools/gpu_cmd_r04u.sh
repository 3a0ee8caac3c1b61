# r04u: cooperative relax parity with the r04s library and with HEAD + the r04t changes (one pass each)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
OUT=gpurun_out/r04u; mkdir -p $OUT
SHDPE_LIB=$R/shadow-1_amd/libshdpe_headt.so timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -k "cooperative" > $OUT/tests_headt.log 2>&1; echo "headt rc=$?"; tail -3 $OUT/tests_headt.log; grep -E "^FAILED" $OUT/tests_headt.log | head
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -k "cooperative" > $OUT/tests_new.log 2>&1; echo "new rc=$?"; tail -3 $OUT/tests_new.log; grep -E "^FAILED" $OUT/tests_new.log | head
true
