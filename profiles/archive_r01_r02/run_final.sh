# round-end evidence: every GPU test, smoke(), the default bench line, rocprof collection
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_all.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_all.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || { tail -20 gpurun_out/bench_final.err; exit 1; }
tail -1 gpurun_out/bench_final.json
bash profiles/collect.sh ${R:-r01n} > gpurun_out/collect.log 2>&1 || { tail -20 gpurun_out/collect.log; exit 1; }
echo collect ok
