# r03: GPU tests given as arguments (default: every -m gpu test), one pytest process
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${T:-600}
timeout -k 10 $T python -u -m pytest ${@:-tests -m gpu} -x -v --timeout 300 --timeout-method thread > gpurun_out/r03_tests.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/r03_tests.log | tail -3; exit $rc
