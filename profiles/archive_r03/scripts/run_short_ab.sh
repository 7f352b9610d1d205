# r03d: the driver's short bench (--steps 20 --warmup 5) vs the default (300 / 20), same box
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for i in 1 2; do
  for a in "--steps 20 --warmup 5" "--steps 300 --warmup 20"; do
    timeout -k 10 200 python -u bench.py --no-cpu-baseline --train-regions 0 --speedy-steps 0 --reservoir-steps 0 $a > gpurun_out/short.json 2> gpurun_out/short.err || { tail -5 gpurun_out/short.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/short.json').read().strip().splitlines()[-1]); print('$a rep $i', d['value'], d['ms_per_step'])"
  done
done
