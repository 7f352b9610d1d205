set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for fz in 1 0; do
SML_DYN_FUSED=$fz timeout -k 10 400 python -u bench.py --no-cpu-baseline --train-regions 0 > gpurun_out/bench_f$fz.json 2> gpurun_out/bench_f$fz.err || exit $?
python3 -c "
import json; d=json.loads(open('gpurun_out/bench_f$fz.json').read().strip().splitlines()[-1])
print('fused=$fz value', d['value'], 'ms', d['ms_per_step'], 'window', d['speedy_step']['window_ms_graph_physics'], d['reservoir_only']['ms_per_step'])"
done
SML_DYN_FUSED=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fprof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --train-regions 0 --reservoir-steps 0 --speedy-steps 8 > gpurun_out/fprof.log 2>&1 || exit $?
python3 - <<'PY'
import csv
r=list(csv.DictReader(open('gpurun_out/fprof/run_kernel_stats.csv')))
for x in r[:14]:
    print(f"{x['Name'][:60]:60s} {int(x['Calls']):6d} {float(x['AverageNs'])/1000:8.2f} {float(x['TotalDurationNs'])/1e6:8.2f}")
PY
