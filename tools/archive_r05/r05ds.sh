# r05ds: the fused path's diagonal-tile update as three 64 x 64 quadrant workgroups (SML_CHOL_DSPLIT=1) vs one lower tile
set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python -u tools/ab_chol_bitwise.py SML_CHOL_FUSE=0 SML_CHOL_DSPLIT=0 SML_CHOL_DSPLIT=1 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r05ds_bitwise.txt || exit 1
bash tools/gpu/ab_train.sh r05ds "SML_CHOL_DSPLIT=0" "SML_CHOL_DSPLIT=1"
