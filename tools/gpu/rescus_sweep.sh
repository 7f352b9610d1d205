#!/bin/bash
# same-box sweep of the reservoir stream's CU count (SML_RES_CUS) at N = 1, alternated
# usage: TAG=r06h bash tools/gpu/rescus_sweep.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
T=${TAG:-r06h}
mkdir -p gpurun_out
B="--no-cpu-baseline --train-regions 0 --reservoir-steps 0 --speedy-steps 0"
for rep in 1 2; do
  for c in 192 160 128; do
    SML_RES_CUS=$c timeout -k 10 300 python -u bench.py $B > gpurun_out/${T}_c${c}_${rep}.json 2> gpurun_out/${T}_c${c}_${rep}.err || exit 1
    python3 -c "import json; d=json.loads(open('gpurun_out/${T}_c${c}_${rep}.json').read().strip().splitlines()[-1]); print('res_cus $c rep $rep', d['value'], d['ms_per_step'], d['roofline']['readout_avg_ms'])"
  done
done
