# reservoir-only bench for several update block splits (experiment)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for p in 1 2 3 4 6; do
SML_UPD_PARTS=$p timeout -k 10 300 python -u bench.py --no-cpu-baseline --train-regions 0 --speedy-steps 0 --steps 5 --warmup 2 --reservoir-steps 30 > gpurun_out/bench_p$p.json 2> gpurun_out/bench_p$p.err || exit $?
python3 -c "
import json; d=json.loads(open('gpurun_out/bench_p$p.json').read().strip().splitlines()[-1])
print('parts $p', 'res_only', d['reservoir_only']['ms_per_step'], 'upd', d['roofline']['update_avg_ms'], 'rd', d['roofline']['readout_avg_ms'])"
done
