# r03d: the update kernel at two 1024-thread blocks per CU (SML_UPD_OCC=2: 64 VGPRs)
# vs one (default), same box: headline + reservoir-only leg
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_reservoir_gpu.py -k "small or full_size or synchronize" > gpurun_out/upd_tests.log 2>&1
rc=$?; tail -1 gpurun_out/upd_tests.log; [ $rc -eq 0 ] || exit $rc
SML_UPD_OCC=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_reservoir_gpu.py -k "small or full_size or synchronize" > gpurun_out/upd_tests2.log 2>&1
rc=$?; tail -1 gpurun_out/upd_tests2.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for e in "X=0" "SML_UPD_OCC=2"; do
    env $e timeout -k 10 200 python -u bench.py --no-cpu-baseline --train-regions 0 --speedy-steps 0 --reservoir-steps 30 > gpurun_out/upd.json 2> gpurun_out/upd.err || { tail -5 gpurun_out/upd.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/upd.json').read().strip().splitlines()[-1]); r=d['roofline']; u=d['reservoir_only']; print('$e rep $i', d['value'], d['ms_per_step'], 'readout', r['readout_avg_ms'], 'update', r['update_avg_ms'], '| res-only', u['value'], u['roofline_unpaced']['update_avg_ms'])"
  done
done
