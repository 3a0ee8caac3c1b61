#!/bin/bash
# Same-box per-rank shard times for several library builds: LIBS="new x y"
# (new = the in-tree libshdpe.so, x -> shadow-1_amd/libshdpe_x.so), workload
# $SHARD_WL at N = $SHARD_NS, REPS rounds alternating; SHDPE_TUNE_LOG=1 prints
# shd_pe_tune's per-variant relax / post times (no kernel counters).
# usage: LIBS="new head" tools/gpu_shard_ab.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
TAG=${1:-r05}; OUT=gpurun_out/$TAG; mkdir -p $OUT
for rep in $(seq 1 ${REPS:-2}); do
  for lib in ${LIBS:-new}; do
    L=$R/shadow-1_amd/libshdpe.so; [ $lib != new ] && L=$R/shadow-1_amd/libshdpe_$lib.so
    SHDPE_LIB=$L SHDPE_TUNE_LOG=1 timeout -k 10 300 python3 -u tools/shard_time.py ${SHARD_WL:-c4} ${SHARD_NS:-8} > $OUT/shardab_$lib.txt 2> $OUT/shardab_$lib.err || { tail -20 $OUT/shardab_$lib.err; exit 1; }
    echo "== $lib #$rep"; cat $OUT/shardab_$lib.txt | sed 's/ \[.*//'; grep "tune" $OUT/shardab_$lib.err
  done
done
