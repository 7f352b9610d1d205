#!/bin/bash
# tools/ab_build.sh REV -- builds libspeedyml.so of git revision REV into ab/REV/
# for same-box A/B measurements (SML_LIB=<printed path> python bench.py ...);
# ab/ is git-ignored and travels to the GPU box with the tree.
set -euo pipefail
REV=$1
ROOT=$(cd "$(dirname "$0")/.." && pwd)
D=$ROOT/ab/$REV
rm -rf "$D"
mkdir -p "$D"
git -C "$ROOT" archive "$REV" speedy-ml-1_amd/csrc include | tar -x -C "$D"
make -C "$D/speedy-ml-1_amd/csrc" -j8 all > "$D/build.log" 2>&1
echo "$D/speedy-ml-1_amd/lib/libspeedyml.so"
