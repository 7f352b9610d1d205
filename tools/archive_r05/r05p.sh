# r05p: 128-row panel tiles (SML_CHOL_PANEL_TILE=128) vs 64
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu/ab_train.sh r05p "SML_CHOL_PANEL_TILE=64" "SML_CHOL_PANEL_TILE=128"
