# r05pre: the update GEMMs starting from their tile (SML_CHOL_PRE=1, default) vs reading it after
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu/ab_train.sh r05pre "SML_CHOL_PRE=0" "SML_CHOL_PRE=1"
