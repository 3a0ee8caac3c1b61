#!/bin/bash
# Build libshdpe.so with extra compiler flags and/or a source patch into
# shadow-1_amd/libshdpe_<name>.so (same-box A/B runs through SHDPE_LIB; the
# in-tree sources and libshdpe.so are untouched: the patch is applied to a
# copy).  Perturbation variants of the batch kernel live in tools/variants/.
# usage: tools/build_variant.sh <name> "<-D flags>" [tools/variants/x.patch]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; FLAGS=$2; PATCH=${3:+$(cd "$(dirname "$3")" && pwd)/$(basename "$3")}
B=/tmp/shdpe_variant_$NAME
rm -rf $B && mkdir -p $B
SRC=$R
if [ -n "$PATCH" ]; then
  SRC=$B/tree; mkdir -p $SRC
  cp -r $R/include $R/shadow-1_amd $SRC/
  rm -rf $SRC/shadow-1_amd/build
  (cd $SRC && patch -s -p1 < "$PATCH")
fi
make -s -C $SRC/shadow-1_amd -j8 B=$B/obj LIB=$B/libshdpe.so HIPFLAGS_EXTRA="$FLAGS" >/dev/null
cp $B/libshdpe.so $R/shadow-1_amd/libshdpe_$NAME.so
echo built shadow-1_amd/libshdpe_$NAME.so with "$FLAGS" ${PATCH:+"+ $PATCH"}
