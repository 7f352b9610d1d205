# Cholesky panel width sweep of the training leg (same box, two reps):
#   bash tools/gpu/panel_sweep.sh <tag> 6 8 10 ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"; tag=$1; shift; o=gpurun_out/$tag; mkdir -p $o
for rep in 1 2; do
  for P in "$@"; do
    f=$o/p${P}_$rep
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --reservoir-steps 0 --speedy-steps 0 --steps 2 --warmup 1 --train-panel $P > $f.json 2> $f.err || { tail $f.err; exit 1; }
    python3 -c "import json; t=json.loads(open('$f.json').read().strip().splitlines()[-1])['training']; print('panel $P rep $rep gram', t['gram_ms'], 'solve', t['solve_ms'], t['solve_roofline']['frac'], t['solve_info_ok'])"
  done
done
