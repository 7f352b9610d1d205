# phase probe of the fused step + default bench (no tests; for A/B experiments)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/probe_phases.py > gpurun_out/probe.log 2>&1 || { tail -20 gpurun_out/probe.log; exit 1; }
cat gpurun_out/probe.log
[ -n "${NO_BENCH:-}" ] && exit 0
timeout -k 10 400 python -u bench.py --no-cpu-baseline --train-regions 0 ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
python3 -c "
import json; d=json.loads(open('gpurun_out/bench.json').read().strip().splitlines()[-1])
print('value', d['value'], 'ms', d['ms_per_step'], 'window', d['speedy_step']['window_ms_graph_physics'], 'res_only', d['reservoir_only']['ms_per_step'])"
