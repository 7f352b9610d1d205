# quick check after a kernel change: hybrid/reservoir GPU tests, a short bench, a rocprof kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/q
timeout -k 10 300 python -u -m pytest tests/test_hybrid_gpu.py tests/test_reservoir_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/q/test.log 2>&1 || { tail -30 gpurun_out/q/test.log; exit 1; }
tail -1 gpurun_out/q/test.log
B="bench.py --no-cpu-baseline --train-regions 0 --reservoir-steps 0 --speedy-steps 0 --steps 50"
for i in 1 2; do
timeout -k 10 200 python -u $B > gpurun_out/q/b$i.json 2> gpurun_out/q/b$i.err || { tail gpurun_out/q/b$i.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/q/b$i.json').read().strip().splitlines()[-1]); print('bench', d['value'], d['ms_per_step'])"
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/q/trace -o trace --output-format csv -- python3 $B --steps 20 > gpurun_out/q/tb.json 2> gpurun_out/q/tb.err || { tail gpurun_out/q/tb.err; exit 1; }
f=$(find gpurun_out/q/trace -name "trace_kernel_stats.csv" | head -1)
python3 -c "
import csv
for x in csv.DictReader(open('$f')):
    if any(k in x['Name'] for k in ('finish', 'assemble', 'tile', 'io_', 'st_inv', 'state_to_m', 'gridx', 'gridy', 'specx', 'specy', 'st_spec', 'st_gridspec')):
        print(f\"{float(x['AverageNs'])/1e3:8.2f} us  {x['Calls']:>5}  {x['Name'][:70]}\")
"
