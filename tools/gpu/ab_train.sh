# Same-box A/B of the training leg over env configurations:
#   bash tools/gpu/ab_train.sh <tag> "A=1 B=0" "A=0 B=0" ...
# training tests once, then two reps of each configuration (solve ms, frac, info ok)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; tag=$1; shift; o=gpurun_out/$tag; mkdir -p $o
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_training_gpu.py > $o/tests.log 2>&1 || { tail -20 $o/tests.log; exit 1; }
tail -1 $o/tests.log
B="bench.py --no-cpu-baseline --reservoir-steps 0 --speedy-steps 0 --steps 2 --warmup 1 ${TRAIN_ARGS:-}"
for rep in 1 2; do
  i=0
  for cfg in "$@"; do
    i=$((i+1)); f=$o/c${i}_$rep
    env $cfg timeout -k 10 400 python -u $B > $f.json 2> $f.err || { tail $f.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); t=d['training']; print('[$cfg] rep $rep gram', t['gram_ms'], 'solve', t['solve_ms'], t['solve_roofline']['frac'], t['solve_info_ok'])"
  done
done
