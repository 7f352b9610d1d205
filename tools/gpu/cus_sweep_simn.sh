set -o pipefail
cd "$GRAFT_REPO_ROOT"; T=${TAG:-r06cs2}; mkdir -p gpurun_out/$T
B="--no-cpu-baseline --train-regions 0 --reservoir-steps 0 --speedy-steps 0"
for rep in 1 2; do
  for cfg in ${CFGS:-"4 192" "4 96" "4 64" "2 192" "2 128"}; do
    set -- $cfg; n=$1; c=$2; f=gpurun_out/$T/n${n}_r${c}_$rep
    SML_RES_CUS=$c timeout -k 10 300 python -u bench.py $B --sim-ranks $n > $f.json 2> $f.err || { tail -3 $f.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); print('sim $n res_cus $c rep $rep', d['value'], d['ms_per_step'])"
  done
done
