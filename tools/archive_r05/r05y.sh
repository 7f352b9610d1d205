# r05y: register diagonal factor with the pivot chain on its own wave -- bitwise, A/B, kernel times
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r05y
timeout -k 10 120 python -u tools/ab_chol_bitwise.py SML_CHOL_DIAG=0 SML_CHOL_DIAG=1 > gpurun_out/r05y/bitwise.log 2>&1 || { tail -20 gpurun_out/r05y/bitwise.log; exit 1; }
grep SML_ gpurun_out/r05y/bitwise.log
bash tools/gpu/prof_train.sh r05y/prof "" && bash tools/gpu/ab_train.sh r05y/ab "SML_CHOL_DIAG=1" "SML_CHOL_DIAG=0"
