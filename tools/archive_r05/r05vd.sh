# r05vd: vdifsc on the longwave side (r05v.sh) and the blocked diagonal factor (ab_train.sh)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu/ab_train.sh r05d2 "SML_CHOL_DIAG=1" "SML_CHOL_DIAG=2" || exit 1
bash tools/gpu/r05v.sh
