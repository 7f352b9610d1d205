# r05af: the solves' wide updates in three right-hand-side groups too -- bitwise, A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r05af
timeout -k 10 120 python -u tools/ab_chol_bitwise.py SML_SOLVE_SPLIT_WIDE=0 SML_SOLVE_SPLIT_WIDE=1 > gpurun_out/r05af/bitwise.log 2>&1 || { tail -20 gpurun_out/r05af/bitwise.log; exit 1; }
grep SML_ gpurun_out/r05af/bitwise.log
bash tools/gpu/ab_train.sh r05af/ab "SML_SOLVE_SPLIT_WIDE=1" "SML_SOLVE_SPLIT_WIDE=0"
