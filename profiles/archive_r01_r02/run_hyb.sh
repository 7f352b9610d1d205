# hybrid-loop change: hybrid / run_model GPU tests, then the default bench line twice (no CPU leg, no training)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_hybrid_gpu.py tests/test_fortran_hybrid_gpu.py tests/test_run_model_gpu.py > gpurun_out/hyb_tests.log 2>&1 || { tail -30 gpurun_out/hyb_tests.log; exit 1; }
tail -1 gpurun_out/hyb_tests.log
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --train-regions 0 --reservoir-steps 0 > gpurun_out/hyb_b$i.json 2> gpurun_out/hyb_b$i.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/hyb_b$i.json')); print('bench', d['value'], d['ms_per_step'], 'window', d['speedy_step']['window_ms_graph_physics'])"
done
