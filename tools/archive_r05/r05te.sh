# r05te: the solves' epilogues through a per-wave LDS transpose (SML_SOLVE_TE=1) vs direct
set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python -u tools/ab_chol_bitwise.py SML_SOLVE_TE=0 SML_SOLVE_TE=1 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r05te2_bitwise.txt || exit 1
bash tools/gpu/ab_train.sh r05te2 "SML_SOLVE_TE=0" "SML_SOLVE_TE=1" || exit 1
bash tools/gpu/prof_train.sh r05tep2 "SML_SOLVE_TE=1" | grep k_solve
