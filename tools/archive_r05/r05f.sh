# r05f: the in-panel update fused with the panel (k_chol_upanel, SML_CHOL_FUSE=1 default) vs two launches
set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python -u tools/ab_chol_bitwise.py SML_CHOL_FUSE=0 SML_CHOL_FUSE=1 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r05f_bitwise.txt || exit 1
bash tools/gpu/ab_train.sh r05f "SML_CHOL_FUSE=0" "SML_CHOL_FUSE=1"
