#!/bin/bash
# r04c: run_model's exit signals the forecast hop in-kernel -- the hybrid tests, then
# a same-box A/B (SML_HOP_FUSED=0: the signal kernel) at N = 1 and in the 8-rank share
set -o pipefail
mkdir -p gpurun_out/r04c
T="timeout -k 10"
$T 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_hybrid_gpu.py tests/test_sharded_gpu.py \
  > gpurun_out/r04c/tests.log 2>&1 || { tail -30 gpurun_out/r04c/tests.log; exit 1; }
tail -3 gpurun_out/r04c/tests.log
B="python -u bench.py --no-cpu-baseline --train-regions 0 --reservoir-steps 0 --speedy-steps 0"
for i in 1 2; do
  for v in A B; do
    if [ $v = A ]; then export SML_HOP_FUSED=0; else unset SML_HOP_FUSED; fi
    $T 240 $B > gpurun_out/r04c/n1_$v$i.json 2> gpurun_out/r04c/n1_$v$i.err || { tail -5 gpurun_out/r04c/n1_$v$i.err; exit 1; }
    $T 240 $B --sim-ranks 8 > gpurun_out/r04c/s8_$v$i.json 2> gpurun_out/r04c/s8_$v$i.err || { tail -5 gpurun_out/r04c/s8_$v$i.err; exit 1; }
    python3 -c "
import json; a=json.load(open('gpurun_out/r04c/n1_$v$i.json')); b=json.load(open('gpurun_out/r04c/s8_$v$i.json'))
print('$v', 'N1', a['value'], a['ms_per_step'], 'sim8', b['value'], b['ms_per_step'])"
  done
done
