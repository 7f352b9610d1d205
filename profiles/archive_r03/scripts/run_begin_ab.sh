# r03d: the fused reservoir begin (k_res_begin, SML_BEGIN=1/2) vs the two-launch
# begin (0): bitwise tests, begin alone / beside the window (probe_contention), and
# same-box A/B of the default bench line, alternated.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_reservoir_gpu.py \
  -k "fused_begin or finish_grid or full_size" > gpurun_out/r03d_tests.log 2>&1 || { tail -30 gpurun_out/r03d_tests.log; exit 1; }
tail -3 gpurun_out/r03d_tests.log
for m in 0 1 2; do
  SML_BEGIN=$m timeout -k 10 240 python -u tools/probe_contention.py > gpurun_out/r03d_contention_$m.log 2>&1 || { tail -5 gpurun_out/r03d_contention_$m.log; exit 1; }
  echo "SML_BEGIN=$m"; cat gpurun_out/r03d_contention_$m.log | grep -E "predict_begin|window"
done
for i in 1 2; do
  for m in 0 1 2; do
    SML_BEGIN=$m timeout -k 10 300 python -u bench.py --no-cpu-baseline --train-regions 0 --speedy-steps 0 --reservoir-steps 0 > gpurun_out/r03d_ab_$m$i.json 2> gpurun_out/r03d_ab_$m$i.err || { tail -5 gpurun_out/r03d_ab_$m$i.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/r03d_ab_$m$i.json').read().strip().splitlines()[-1]); r=d['roofline']; print('SML_BEGIN=$m rep $i', d['value'], d['ms_per_step'], r['readout_avg_ms'], r['update_avg_ms'], r['frac'])"
  done
done
