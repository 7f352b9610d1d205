#!/bin/bash
# same-box sweep of the CU split in the 8-rank share (--sim-ranks 8), alternated:
#   SPEEDY's CUs (--speedy-cus) and the reservoir stream's (SML_RES_CUS)
# usage: TAG=r06cs bash tools/gpu/cus_sweep_sim8.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
T=${TAG:-r06cs}
mkdir -p gpurun_out/$T
B="--no-cpu-baseline --train-regions 0 --reservoir-steps 0 --speedy-steps 0 --sim-ranks 8"
for rep in 1 2; do
  for cfg in "64 192" "48 208" "96 160" "128 128" "64 128" "64 64"; do
    set -- $cfg; s=$1; c=$2; f=gpurun_out/$T/s${s}_r${c}_$rep
    SML_RES_CUS=$c timeout -k 10 300 python -u bench.py $B --speedy-cus $s > $f.json 2> $f.err || { tail -3 $f.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); print('speedy_cus $s res_cus $c rep $rep', d['value'], d['ms_per_step'])"
  done
done
