# fused-step GPU tests, then the phase probe + bench for the merged grid kernel and the split form
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_physics_gpu.py tests/test_spectral_gpu.py tests/test_reservoir_gpu.py tests/test_hybrid_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -5 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
bash profiles/run_probe.sh || exit $?
echo "--- split grid"
SML_DYN_SPLIT_GRID=1 bash profiles/run_probe.sh
