# r05k: evidence at the final round-5 defaults (fused in-panel update, quadrant diagonal-tile update, transposed epilogues) (tests, smoke, bench, driver command, rocprof)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=r05k bash tools/gpu/evidence.sh
