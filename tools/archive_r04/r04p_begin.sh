#!/bin/bash
# r04p: the begin's form re-measured with the compressed update (SML_BEGIN: 0 the
# update grid then the readout grid, 1 / 2 one fused launch) -- same-box A/B/C
set -o pipefail
mkdir -p gpurun_out/r04p
T="timeout -k 10"
B="python -u bench.py --no-cpu-baseline --train-regions 0 --reservoir-steps 0 --speedy-steps 0"
for i in 1 2 3; do
  for v in 0 1; do
    SML_BEGIN=$v $T 300 $B > gpurun_out/r04p/b$v-$i.json 2> gpurun_out/r04p/b$v-$i.err || { tail -5 gpurun_out/r04p/b$v-$i.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/r04p/b$v-$i.json').read().strip().splitlines()[-1])
print('begin $v', d['value'], d['ms_per_step'])"
  done
done
