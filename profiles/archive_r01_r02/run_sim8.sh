# diagnostic: rank 0's share of an 8-rank run on one GPU, one stream vs overlap
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for n in ${SIMS:-8}; do for ov in "--no-overlap" "--overlap"; do
timeout -k 10 300 python -u bench.py --sim-ranks $n --no-cpu-baseline --train-regions 0 --speedy-steps 0 --reservoir-steps 20 $ov > gpurun_out/sim$n$ov.json 2> gpurun_out/sim$n$ov.err || { tail -5 gpurun_out/sim$n$ov.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/sim$n$ov.json').read().strip().splitlines()[-1])
print('sim$n $ov value', d['value'], 'ms', d['ms_per_step'], 'res_only', d['reservoir_only']['ms_per_step'], 'rd', d['roofline']['readout_avg_ms'], 'upd', d['roofline']['update_avg_ms'])"
done; done
