# r05ct: the factor's shallow launches with the transposed epilogue (SML_CHOL_TE=1) vs direct; training tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python -u tools/ab_chol_bitwise.py SML_CHOL_TE=0 SML_CHOL_TE=1 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r05ct_bitwise.txt || exit 1
bash tools/gpu/ab_train.sh r05ct "SML_CHOL_TE=0" "SML_CHOL_TE=1" || exit 1
bash tools/gpu/prof_train.sh r05ctp "" | grep k_chol
