# r03d: --sim-ranks N (rank 0's share of an N-rank decomposition, the all-gather a
# local copy: a diagnostic of the per-rank step, never the headline)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for n in 1 2 4 8; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --train-regions 0 --speedy-steps 0 --reservoir-steps 0 --sim-ranks $n > gpurun_out/sim$n.json 2> gpurun_out/sim$n.err || { tail -5 gpurun_out/sim$n.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/sim$n.json').read().strip().splitlines()[-1]); print('sim-ranks $n', d['value'], d['ms_per_step'])"
done
