# r04h: HEAD profile set (full GPU suite, driver-default bench, rocprof trace + PMC traffic for C4,
# trace of C3a / C5 / C2) and a C2 sparse-kernel knob sweep
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
OUT=gpurun_out/r04h; mkdir -p $OUT
STAGES="tests default trace pmc" WLS=c4 bash tools/gpu_r04.sh r04h || exit 1
STAGES="trace" WLS=c3a,c5,c2 bash tools/gpu_r04.sh r04h || exit 1
QUICK='--no-cpu --tie-stress= --secondary= --host-fill 0 --d2h-rows 0 --no-stream'
for e in "X=0" "SHDPE_DELTA_FACTOR=8" "SHDPE_DELTA_FACTOR=24" "SHDPE_DELTA_FACTOR=32" "SHDPE_KFLAGS=16" "SHDPE_KFLAGS=48" "SHDPE_THREADS=256" "SHDPE_THREADS=1024" "SHDPE_HEAVY_DEG=32"; do
  env $e timeout -k 10 200 python3 -u bench.py --workload c2 --steps 5 --warmup 1 $QUICK > $OUT/c2_$e.json 2> $OUT/c2_$e.err || { tail -5 $OUT/c2_$e.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/c2_$e.json')); print('c2 $e', round(d['ms_per_step'],2), 'ms', round(d['roofline']['frac'],4))"
done
