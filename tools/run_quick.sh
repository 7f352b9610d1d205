# quick check after a change: hybrid/reservoir GPU tests, short benches (1 GPU and the simulated 2/8-rank shares)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/q
timeout -k 10 300 python -u -m pytest tests/test_hybrid_gpu.py tests/test_reservoir_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/q/test.log 2>&1 || { tail -30 gpurun_out/q/test.log; exit 1; }
tail -1 gpurun_out/q/test.log
B="bench.py --no-cpu-baseline --train-regions 0 --reservoir-steps 0 --speedy-steps 0 --steps 50"
for v in "1" "2" "s2 --sim-ranks 2" "s8 --sim-ranks 8" "s8n --sim-ranks 8 --speedy-cus 0"; do
set -- $v; name=$1; shift
timeout -k 10 200 python -u $B "$@" > gpurun_out/q/b$name.json 2> gpurun_out/q/b$name.err || { tail gpurun_out/q/b$name.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/q/b$name.json').read().strip().splitlines()[-1]); print('bench $name', d['value'], d['ms_per_step'], d['roofline']['achieved'], d['roofline']['readout_avg_ms'])"
done
