# r05sp: the triangular solves' panel width (SML_SOLVE_PANEL) 8 (the factor's) / 6 / 4 / 3; training tests under 4
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r05sp
SML_SOLVE_PANEL=4 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_training_gpu.py > gpurun_out/r05sp/tests_sp4.log 2>&1 || { tail -20 gpurun_out/r05sp/tests_sp4.log; exit 1; }
tail -1 gpurun_out/r05sp/tests_sp4.log
timeout -k 10 200 python -u tools/ab_chol_bitwise.py SML_SOLVE_PANEL=8 SML_SOLVE_PANEL=4 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r05sp/bitwise.txt || exit 1
bash tools/gpu/ab_train.sh r05sp "SML_SOLVE_PANEL=8" "SML_SOLVE_PANEL=6" "SML_SOLVE_PANEL=4" "SML_SOLVE_PANEL=3"
