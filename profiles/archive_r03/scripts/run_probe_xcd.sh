set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 tools/probe_xcd_l2 ${LAYOUT:-} 2>&1 | tee gpurun_out/probe_xcd_l2.log
