# r05s: cleaned training solve (right-hand-side split + LDS-transposed W_out) -- tests, bitwise, A/B, kernel times
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r05s
timeout -k 10 120 python -u tools/ab_chol_bitwise.py SML_SOLVE_SPLIT=0 SML_SOLVE_SPLIT=1 > gpurun_out/r05s/bitwise.log 2>&1 || { tail -20 gpurun_out/r05s/bitwise.log; exit 1; }
grep SML_ gpurun_out/r05s/bitwise.log
bash tools/gpu/ab_train.sh r05s/ab "SML_SOLVE_SPLIT=1" "SML_SOLVE_SPLIT=0" && bash tools/gpu/prof_train.sh r05s/prof ""
