# Same-box A/B of the default bench (N = 1 and the 8-rank share) over env configurations:
#   bash tools/gpu/ab_bench.sh <tag> "A=1" "A=0" ...   (two alternations of each)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; tag=$1; shift; o=gpurun_out/$tag; mkdir -p $o
for rep in 1 2; do
  i=0
  for cfg in "$@"; do
    i=$((i+1))
    for sim in 1 8; do
      f=$o/c${i}_s${sim}_$rep
      env $cfg timeout -k 10 300 python -u bench.py --no-cpu-baseline --train-regions 0 --sim-ranks $sim > $f.json 2> $f.err || { tail $f.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); print('[$cfg] sim $sim rep $rep', d['value'], d['ms_per_step'])"
    done
  done
done
