set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests/test_window_ref_gpu.py tests/test_full_size_gpu.py -v -s --timeout 600 --timeout-method thread > gpurun_out/r02c_tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|err per field|assert" gpurun_out/r02c_tests.log | head -40; exit $rc
