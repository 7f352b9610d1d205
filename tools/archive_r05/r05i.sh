# r05i: evidence at the fused in-panel update default (tests, smoke, bench, driver command, rocprof)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=r05i bash tools/gpu/evidence.sh
