set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r06sp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_run_model_gpu.py tests/test_hybrid_gpu.py > gpurun_out/r06sp/tests.log 2>&1 || { tail -20 gpurun_out/r06sp/tests.log; exit 1; }
tail -1 gpurun_out/r06sp/tests.log
B="--no-cpu-baseline --train-regions 0 --reservoir-steps 0 --speedy-steps 0"
for sim in 1 8; do
  f=gpurun_out/r06sp/sim$sim
  timeout -k 10 300 python -u bench.py $B --sim-ranks $sim > $f.json 2> $f.err || { tail -3 $f.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); print('sim $sim', d['value'], d['run_speedy_poll']['value_without_poll'], d['run_speedy_poll']['cost_pct'])"
done
cat /proc/loadavg
