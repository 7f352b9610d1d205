# overlapped hybrid step vs the v_ml readout's wave cap (SML_READ_WAVES)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for w in ${WAVES:-0 4096 2048 1024 512}; do
SML_READ_WAVES=$w timeout -k 10 300 python -u bench.py --no-cpu-baseline --train-regions 0 --speedy-steps 0 --reservoir-steps 0 > gpurun_out/rw$w.json 2> gpurun_out/rw$w.err || { tail -5 gpurun_out/rw$w.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/rw$w.json').read().strip().splitlines()[-1])
print('read_waves $w value', d['value'], 'ms', d['ms_per_step'], 'rd', d['roofline']['readout_avg_ms'], 'upd', d['roofline']['update_avg_ms'])"
done
