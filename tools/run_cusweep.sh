set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/cus
timeout -k 10 200 python -u -m pytest tests/test_hybrid_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/cus/test.log 2>&1 || { tail -30 gpurun_out/cus/test.log; exit 1; }
tail -1 gpurun_out/cus/test.log
for c in 64 0 80 96 64 0 72; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --train-regions 0 --reservoir-steps 0 --speedy-steps 0 --steps 50 --speedy-cus $c > gpurun_out/cus/b$c.json 2> gpurun_out/cus/b$c.err || { tail gpurun_out/cus/b$c.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/cus/b$c.json').read().strip().splitlines()[-1]); print($c, d['value'], d['ms_per_step'])"
done
