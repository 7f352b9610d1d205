# r03: GPU tests named in $TESTS, then the default bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 ${T:-600} python -u -m pytest $TESTS -x -v --timeout 300 --timeout-method thread > gpurun_out/r03_tests.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/r03_tests.log | tail -3; [ $rc -eq 0 ] || exit $rc
OUT=${OUT:-r03_bench}
timeout -k 10 900 python -u bench.py $BENCH_ARGS > gpurun_out/$OUT.json 2> gpurun_out/$OUT.err
rc=$?; tail -2 gpurun_out/$OUT.err; exit $rc
