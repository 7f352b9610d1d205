# r05x: the triangular solves' launches as XCD-grouped 1-D grids (SML_SOLVE_XCD=1) vs 3-D grids; training tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python -u tools/ab_chol_bitwise.py SML_SOLVE_XCD=0 SML_SOLVE_XCD=1 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r05x_bitwise.txt || exit 1
bash tools/gpu/ab_train.sh r05x "SML_SOLVE_XCD=0" "SML_SOLVE_XCD=1" || exit 1
SML_SOLVE_XCD=1 bash tools/gpu/prof_train.sh r05xp "" | tail -14
