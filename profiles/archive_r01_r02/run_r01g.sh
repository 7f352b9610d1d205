set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v -x --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log; tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
echo bench ok
export TMPDIR=/tmp
SML_DYN_UNFUSED=1 timeout -k 10 400 python -u bench.py > gpurun_out/bench_unfused.json 2> gpurun_out/bench_unfused.err || exit $?
echo bench unfused ok
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r01g -o run -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/prof.log 2>&1 || exit $?
echo prof ok
