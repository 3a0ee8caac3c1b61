#!/bin/bash
# Build libshdpe.so from a git revision (default HEAD) into
# shadow-1_amd/libshdpe_head.so for same-box A/B runs (SHDPE_LIB).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
REV=${1:-HEAD}
W=/tmp/shdpe_head_tree
rm -rf $W && mkdir -p $W
git -C $R archive $REV shadow-1_amd include | tar -x -C $W
make -s -C $W/shadow-1_amd -j8 >/dev/null
cp $W/shadow-1_amd/libshdpe.so $R/shadow-1_amd/libshdpe_head.so
echo "built shadow-1_amd/libshdpe_head.so from $(git -C $R rev-parse --short $REV)"
