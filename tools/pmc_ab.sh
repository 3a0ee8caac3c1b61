#!/bin/bash
# PMC passes (one counter group per run) on one workload for the HEAD build
# (libshdpe_head.so) and the working build (libshdpe.so): L2-miss traffic,
# L2 hit rate and L2 atomics of the dominant kernel.
# usage: tools/pmc_ab.sh <workload> <outdir>
set -o pipefail
WL=${1:-c4}; OUT=${2:-gpurun_out/pmc}
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/$OUT
cd /tmp && export TMPDIR=/tmp
for lib in head new; do
  L=$R/shadow-1_amd/libshdpe.so; [ $lib = head ] && L=$R/shadow-1_amd/libshdpe_head.so
  for PASS in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" ${EXTRA_PASSES}; do
    TAG=$(echo $PASS | tr ' ' '_' | cut -c1-40)
    SHDPE_LIB=$L timeout -s KILL 150 rocprofv3 --pmc $PASS --output-format csv -d $R/$OUT/${lib}_$TAG -o pmc -- python3 $R/tools/prof_run.py $WL 1 > $R/$OUT/${lib}_$TAG.log 2>&1 || { echo "pass $lib $PASS failed"; tail -5 $R/$OUT/${lib}_$TAG.log; exit 1; }
  done
done
python3 - "$R/$OUT" <<'PY'
import csv, glob, os, sys
from collections import defaultdict
root = sys.argv[1]
for lib in ("head", "new"):
    tot = defaultdict(float)
    for f in glob.glob(os.path.join(root, lib + "_*", "**", "*counter_collection*.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "batch" in r.get("Kernel_Name", "") or "sparse" in r.get("Kernel_Name", ""):
                tot[r["Counter_Name"]] += float(r["Counter_Value"])
    fs, ws = tot.get("FETCH_SIZE", 0) * 1024, tot.get("WRITE_SIZE", 0) * 1024
    h, m = tot.get("TCC_HIT_sum", 0), tot.get("TCC_MISS_sum", 0)
    print(lib, f"fetch(x2)={2*fs/1e9:.1f} GB write={ws/1e9:.1f} GB total={(2*fs+ws)/1e9:.1f} GB  L2 hit={h/max(h+m,1):.3f}",
          " ".join(f"{k}={v:.4g}" for k, v in sorted(tot.items()) if k not in ("FETCH_SIZE", "WRITE_SIZE", "TCC_HIT_sum", "TCC_MISS_sum")))
PY
