# overlapped hybrid step vs the paced update's grid cap (SML_UPD_BLOCKS)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for b in ${BLOCKS:-0 256 128 64}; do
SML_UPD_BLOCKS=$b timeout -k 10 300 python -u bench.py --no-cpu-baseline --train-regions 0 --speedy-steps 0 --reservoir-steps 0 > gpurun_out/ub$b.json 2> gpurun_out/ub$b.err || { tail -5 gpurun_out/ub$b.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/ub$b.json').read().strip().splitlines()[-1])
print('upd_blocks $b value', d['value'], 'ms', d['ms_per_step'], 'rd', d['roofline']['readout_avg_ms'], 'upd', d['roofline']['update_avg_ms'])"
done
