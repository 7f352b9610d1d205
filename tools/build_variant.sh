#!/bin/bash
# tools/build_variant.sh NAME [make variables...] -- builds the WORKING TREE's
# libspeedyml.so with extra flags into abx/NAME/ (git-ignored, but shipped to the GPU
# box with the tree): e.g. a profiling build,
#   bash tools/build_variant.sh pst 'FLAGS_sml_dynamics=-ffp-contract=on -DSML_PSTAMPS'
# then SML_LIB=abx/NAME/speedy-ml-1_amd/lib/libspeedyml.so python ...
set -euo pipefail
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
D=$ROOT/abx/$NAME
rm -rf "$D"
mkdir -p "$D/speedy-ml-1_amd"
cp -r "$ROOT/speedy-ml-1_amd/csrc" "$D/speedy-ml-1_amd/"
cp -r "$ROOT/include" "$D/"
make -C "$D/speedy-ml-1_amd/csrc" -j8 "$@" "$D/speedy-ml-1_amd/lib/libspeedyml.so" > "$D/build.log" 2>&1 || { tail -20 "$D/build.log"; exit 1; }
echo "$D/speedy-ml-1_amd/lib/libspeedyml.so"
