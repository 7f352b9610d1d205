# reservoir / hybrid GPU tests, then overlap + serial benches
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_reservoir_gpu.py tests/test_hybrid_gpu.py tests/test_exchange_gpu.py tests/test_fortran_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -5 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
SIMS="1" bash profiles/run_sim8.sh
