set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
T=${1:-r06m}; mkdir -p gpurun_out/$T
for w in 0 4 8; do
  SHDPE_TUNE_FAIL_WPE=$w SHDPE_TUNE_LOG=1 timeout -k 10 120 python3 -u tools/tune_fail_probe.py > gpurun_out/$T/probe_$w.txt 2> gpurun_out/$T/probe_$w.err || { tail -5 gpurun_out/$T/probe_$w.err; exit 1; }
  echo "== fail wpe $w"; cat gpurun_out/$T/probe_$w.txt; grep "tune" gpurun_out/$T/probe_$w.err
done
