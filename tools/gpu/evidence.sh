#!/bin/bash
# evidence at HEAD: the full -m gpu suite, smoke(), the default bench line, the
# driver's own command, then the rocprofv3 summary (profiles/collect.sh)
# usage: TAG=r04d bash tools/gpu/evidence.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
T=${TAG:-r04d}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/${T}_gpu_tests.log | tail -2; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1
rc=$?; tail -1 gpurun_out/${T}_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
rc=$?; tail -2 gpurun_out/${T}_bench.err; [ $rc -eq 0 ] || exit $rc
python3 -c "import json; d=json.loads(open('gpurun_out/${T}_bench.json').read().strip().splitlines()[-1]); r=d['roofline']; print(d['value'], d['ms_per_step'], r['frac'], 'update', r['update_avg_ms'], d['speedy_step']['window_ms_graph_physics'])"
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${T}_bench_driver.json 2> gpurun_out/${T}_bench_driver.err || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/${T}_bench_driver.json').read().strip().splitlines()[-1]); print('driver-style', d['value'], d['ms_per_step'])"
[ "${PROF:-1}" = 1 ] || exit 0
bash profiles/collect.sh $T
