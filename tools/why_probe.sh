#!/bin/bash
# Why did a batch's rows leave the fast path?  The test_batched_kernel_each_lb
# power-law case at LB 4 / 8 waves through each library build in $LIBS (new =
# in-tree libshdpe.so, else shadow-1_amd/libshdpe_<x>.so; diag builds carry
# -DSHDPE_DIAG_WHY and print the per-reason batch counts).
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
OUT=gpurun_out/${1:-why}; mkdir -p $OUT
for lib in ${LIBS:-new diag}; do
  L=shadow-1_amd/libshdpe.so; [ $lib != new ] && L=shadow-1_amd/libshdpe_$lib.so
  SHDPE_LIB=$R/$L SHDPE_DEBUG=1 SHDPE_BATCH_LB=${LB:-4} SHDPE_BATCH_WPE=${WPE:-8} timeout -k 10 120 \
    python3 -u tools/lb8_probe.py rows > $OUT/why_$lib.txt 2> $OUT/why_$lib.err || { echo "$lib failed"; tail -5 $OUT/why_$lib.err; exit 1; }
  echo "== $lib"; cat $OUT/why_$lib.txt; grep -E "batch why|tie batches" $OUT/why_$lib.err | sort | uniq -c | head -6
done
