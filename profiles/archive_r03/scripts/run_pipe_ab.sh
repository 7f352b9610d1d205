# r03d: the pipelined loop (default now) vs --no-pipelined at the driver's 20 / 5 and
# at 300 / 20, same box; the hybrid tests first
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_hybrid_gpu.py tests/test_fortran_hybrid_gpu.py > gpurun_out/pipe_tests.log 2>&1
rc=$?; tail -1 gpurun_out/pipe_tests.log; [ $rc -eq 0 ] || { tail -30 gpurun_out/pipe_tests.log; exit $rc; }
for i in 1 2; do
  for a in "--steps 20 --warmup 5" "--steps 20 --warmup 5 --no-pipelined" "--steps 300 --warmup 20" "--steps 300 --warmup 20 --no-pipelined"; do
    timeout -k 10 200 python -u bench.py --no-cpu-baseline --train-regions 0 --speedy-steps 0 --reservoir-steps 5 $a > gpurun_out/pipe.json 2> gpurun_out/pipe.err || { tail -5 gpurun_out/pipe.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/pipe.json').read().strip().splitlines()[-1]); print('$a rep $i', d['value'], d['ms_per_step'], d['roofline']['readout_avg_ms'], d['roofline']['update_avg_ms'])"
  done
done
