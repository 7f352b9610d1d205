set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_reservoir_gpu.py tests/test_hybrid_gpu.py tests/test_full_size_gpu.py -v -s --timeout 600 --timeout-method thread > gpurun_out/r02e_tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|configs\[2\] after|assert" gpurun_out/r02e_tests.log | head -60; exit $rc
