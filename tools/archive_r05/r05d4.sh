# r05d4: the register sub-block factor in k_chol_diag_b -- training tests, A/B vs k_chol_diag, kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu/ab_train.sh r05d4 "SML_CHOL_DIAG=1" "SML_CHOL_DIAG=2" || exit 1
bash tools/gpu/prof_train.sh r05d4p "SML_CHOL_DIAG=2"
