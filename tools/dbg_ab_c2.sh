#!/bin/bash
# Same-box A/B of k_sparse_rows per-row cycle counters (SHDPE_DEBUG) on C2:
# LIBS="new x" -> in-tree libshdpe.so vs shadow-1_amd/libshdpe_x.so
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; OUT=gpurun_out/${1:-dbgab}; mkdir -p $OUT
Q='--workload c2 --steps 3 --warmup 1 --no-cpu --tie-stress= --secondary= --host-fill 0 --d2h-rows 0 --no-stream'
for rep in 1 2; do
  for lib in ${LIBS:-new}; do
    L=shadow-1_amd/libshdpe.so; [ $lib != new ] && L=shadow-1_amd/libshdpe_$lib.so
    SHDPE_LIB=$R/$L SHDPE_DEBUG=1 timeout -k 10 200 python3 -u bench.py $Q > $OUT/$lib.json 2> $OUT/$lib.err || { tail -5 $OUT/$lib.err; exit 1; }
    echo "$lib #$rep $(grep 'sparse rows' $OUT/$lib.err | tail -1 | sed 's/.*kcycles/kcycles/')"
  done
done
