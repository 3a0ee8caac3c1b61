set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out/r06b
for v in r5 pf5; do
  SHDPE_LIB=$PWD/shadow-1_amd/libshdpe_$v.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -k "test_batched_kernel_each_lb" -v --timeout 120 --timeout-method thread > gpurun_out/r06b/each_lb_$v.log 2>&1
  echo "== $v rc=$?"; grep -E "PASS|FAIL" gpurun_out/r06b/each_lb_$v.log | sed 's/.*::/  /' | head -20
done
LIBS="r5 pf5" tools/why_probe.sh r06b || exit 1
WLS=c3b ENVS="SHDPE_PRED_MI=2;SHDPE_PRED_MI=3;SHDPE_PRED_MI=2;SHDPE_PRED_MI=3" STEPS=1 STAGES=envs tools/gpu_r05.sh r06b
