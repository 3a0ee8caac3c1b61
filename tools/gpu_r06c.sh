# r05au reproduction on the tree the variant was measured on (6ce98cf), and
# the blockIdx -> XCD placement of persistent grids (tools/micro/xcc_probe)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out/r06c
for g in "256 1024" "512 1024" "512 768" "1024 256"; do timeout -k 10 60 tools/micro/xcc_probe $g || exit 1; done
for v in au pfau; do
  SHDPE_LIB=$PWD/shadow-1_amd/libshdpe_$v.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -k "test_batched_kernel_each_lb" -v --timeout 120 --timeout-method thread > gpurun_out/r06c/each_lb_$v.log 2>&1
  echo "== $v rc=$?"; grep -E "PASS|FAIL" gpurun_out/r06c/each_lb_$v.log | sed 's/.*::/  /' | head -20
  grep -E "^E .*(assert|rowsExact)" gpurun_out/r06c/each_lb_$v.log | head -5
done
LIBS="au pfau" tools/why_probe.sh r06c
