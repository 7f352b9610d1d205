set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_fortran_hybrid_gpu.py tests/test_hybrid_gpu.py -x -v --timeout 400 --timeout-method thread > gpurun_out/r02b_tests.log 2>&1
rc=$?; tail -15 gpurun_out/r02b_tests.log; exit $rc
