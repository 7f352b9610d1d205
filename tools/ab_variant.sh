#!/bin/bash
# tools/ab_variant.sh NAME "DEFINES" -- builds the working tree's libspeedyml.so with
# extra compile definitions for sml_dynamics.hip (e.g. "-DSML_LW_FB_GLOBAL") into
# ab/NAME/ for same-box A/B runs (SML_LIB=<printed path>); ab/ is git-ignored.
set -euo pipefail
NAME=$1
DEFS=${2:-}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
D=$ROOT/ab/$NAME
rm -rf "$D"
mkdir -p "$D/speedy-ml-1_amd"
cp -r "$ROOT/speedy-ml-1_amd/csrc" "$D/speedy-ml-1_amd/"
cp -r "$ROOT/include" "$D/"
make -C "$D/speedy-ml-1_amd/csrc" -j8 all FLAGS_sml_dynamics="-ffp-contract=on $DEFS" > "$D/build.log" 2>&1
echo "$D/speedy-ml-1_amd/lib/libspeedyml.so"
