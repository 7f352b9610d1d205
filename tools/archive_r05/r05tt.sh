# r05tt: the trailing update with the transposed epilogue (SML_CHOL_TE_TRAIL=1) vs direct
set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python -u tools/ab_chol_bitwise.py SML_CHOL_TE_TRAIL=0 SML_CHOL_TE_TRAIL=1 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r05tt_bitwise.txt || exit 1
bash tools/gpu/ab_train.sh r05tt "SML_CHOL_TE_TRAIL=0" "SML_CHOL_TE_TRAIL=1" || exit 1
bash tools/gpu/prof_train.sh r05ttp "SML_CHOL_TE_TRAIL=1" | grep k_chol_update
