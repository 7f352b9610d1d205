# r03d evidence at HEAD: the full -m gpu suite, smoke(), then the default bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG:-r03d}_gpu_tests.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/${TAG:-r03d}_gpu_tests.log | tail -2; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG:-r03d}_smoke.log 2>&1
rc=$?; tail -1 gpurun_out/${TAG:-r03d}_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u bench.py > gpurun_out/${TAG:-r03d}_bench.json 2> gpurun_out/${TAG:-r03d}_bench.err
rc=$?; tail -2 gpurun_out/${TAG:-r03d}_bench.err; python3 -c "import json; d=json.loads(open('gpurun_out/${TAG:-r03d}_bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['speedy_step']['window_ms_graph_physics'])"; [ $rc -eq 0 ] || exit $rc
# the driver's own command (20 timed steps after 5 warm-up)
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG:-r03d}_bench_driver.json 2> gpurun_out/${TAG:-r03d}_bench_driver.err || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/${TAG:-r03d}_bench_driver.json').read().strip().splitlines()[-1]); print('driver-style', d['value'], d['ms_per_step'])"
