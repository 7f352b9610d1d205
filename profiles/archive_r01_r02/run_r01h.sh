# GPU tests, bench (overlapped and single-stream), rocprof trace + PMC for round r01h
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v -x --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log; tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
echo bench ok
timeout -k 10 400 python -u bench.py --no-overlap --no-cpu-baseline --train-regions 0 > gpurun_out/bench_serial.json 2> gpurun_out/bench_serial.err || exit $?
echo bench serial ok
timeout -k 10 900 bash profiles/collect.sh r01h > gpurun_out/collect.log 2>&1 || exit $?
echo collect ok
