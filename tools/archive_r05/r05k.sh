# r05k: the trailing update's LDS stage depth 32 (SML_CHOL_KC=32) vs 16
set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python -u tools/ab_chol_bitwise.py SML_CHOL_FUSE=0 SML_CHOL_KC=32 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r05k_bitwise.txt || exit 1
bash tools/gpu/ab_train.sh r05k "SML_CHOL_KC=16" "SML_CHOL_KC=32"
