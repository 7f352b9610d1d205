# window + headline after a SPEEDY kernel change: dynamics / physics / run_model GPU tests, then bench (no training, no CPU leg)
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
timeout -k 10 400 $T tests/test_dynamics_gpu.py tests/test_physics_gpu.py tests/test_run_model_gpu.py tests/test_window_ref_gpu.py > gpurun_out/win_tests.log 2>&1 || { tail -30 gpurun_out/win_tests.log; exit 1; }
tail -2 gpurun_out/win_tests.log
B="python -u bench.py --steps 300 --warmup 10 --no-cpu-baseline --train-regions 0 --reservoir-steps 0"
for i in 1 2; do
  timeout -k 10 200 $B > gpurun_out/win_b$i.json 2> gpurun_out/win_b$i.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/win_b$i.json')); s=d.get('speedy_step',{}); print('bench', d['value'], d['ms_per_step'], 'window', s.get('window_ms_graph_physics'))"
done
