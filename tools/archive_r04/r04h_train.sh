#!/bin/bash
# r04h: + the diagonal update tiles skip the wave above the diagonal -- the training tests, then
# A (the previous build) / B (this tree) on the bench's training leg
set -o pipefail
mkdir -p gpurun_out/r04h
T="timeout -k 10"
$T 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_training_gpu.py \
  > gpurun_out/r04h/tests.log 2>&1 || { tail -30 gpurun_out/r04h/tests.log; exit 1; }
tail -1 gpurun_out/r04h/tests.log
B="python -u bench.py --no-cpu-baseline --steps 2 --warmup 1 --reservoir-steps 0 --speedy-steps 0"
for i in 1 2; do
  for v in A B; do
    unset SML_LIB; [ $v = A ] && export SML_LIB=$PWD/ablib/libspeedyml_0edeac5.so
    $T 300 $B > gpurun_out/r04h/t_$v$i.json 2> gpurun_out/r04h/t_$v$i.err || { tail -5 gpurun_out/r04h/t_$v$i.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/r04h/t_$v$i.json').read().strip().splitlines()[-1]); t=d['training']
print('$v', 'gram_ms', t['gram_ms'], t['roofline']['achieved'], t['roofline']['frac'], 'solve_ms', t['solve_ms'], t['solve_roofline']['achieved'], t['solve_roofline']['frac'], 'ok', t['solve_info_ok'])"
  done
done
