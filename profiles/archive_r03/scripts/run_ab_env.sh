# r03: same-box A/B of the default bench line under two environments:
#   A_ENV / B_ENV (e.g. "SML_WOUT_MEM=uncached"), alternated REPS times
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for i in $(seq 1 ${REPS:-2}); do
  for arm in A B; do
    envs=$([ $arm = A ] && echo "$A_ENV" || echo "$B_ENV")
    env $envs timeout -k 10 300 python -u bench.py --no-cpu-baseline --train-regions 0 --speedy-steps 0 --reservoir-steps 0 $BENCH_ARGS > gpurun_out/ab_$arm$i.json 2> gpurun_out/ab_$arm$i.err || { tail -5 gpurun_out/ab_$arm$i.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/ab_$arm$i.json').read().strip().splitlines()[-1]); print('$arm$i', '$envs', d['value'], d['ms_per_step'], d['roofline']['frac'])"
  done
done
