#!/bin/bash
# Build libshdpe.so with extra compiler flags into shadow-1_amd/libshdpe_<name>.so
# (same-box A/B runs through SHDPE_LIB; the in-tree libshdpe.so is untouched).
# usage: tools/build_variant.sh <name> "<-D flags>"
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; FLAGS=$2
B=/tmp/shdpe_variant_$NAME
rm -rf $B && mkdir -p $B
make -s -C $R/shadow-1_amd -j8 B=$B LIB=$B/libshdpe.so HIPFLAGS_EXTRA="$FLAGS" >/dev/null
cp $B/libshdpe.so $R/shadow-1_amd/libshdpe_$NAME.so
echo built shadow-1_amd/libshdpe_$NAME.so with "$FLAGS"
