#!/bin/bash
# r04d: the balanced update with pass-uniform branches (no zero-byte loads) at depth 2
# and 3 -- the ELL tests, then A (HEAD's layout) / B (depth 2) / C (depth 3)
set -o pipefail
mkdir -p gpurun_out/r04d
T="timeout -k 10"
$T 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_reservoir_gpu.py \
  -k "ell_layouts or balanced" > gpurun_out/r04d/tests.log 2>&1 || { tail -30 gpurun_out/r04d/tests.log; exit 1; }
SML_UPD_DEPTH=3 $T 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_reservoir_gpu.py \
  -k "ell_layouts or balanced" > gpurun_out/r04d/tests_d3.log 2>&1 || { tail -30 gpurun_out/r04d/tests_d3.log; exit 1; }
tail -1 gpurun_out/r04d/tests.log; tail -1 gpurun_out/r04d/tests_d3.log
B="python -u bench.py --no-cpu-baseline --train-regions 0 --speedy-steps 0"
for i in 1 2; do
  for v in A B C; do
    unset SML_LIB SML_UPD_DEPTH
    [ $v = A ] && export SML_LIB=$PWD/ablib/libspeedyml_head.so
    [ $v = C ] && export SML_UPD_DEPTH=3
    $T 240 $B > gpurun_out/r04d/ab_$v$i.json 2> gpurun_out/r04d/ab_$v$i.err || { tail -5 gpurun_out/r04d/ab_$v$i.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/r04d/ab_$v$i.json')); r=d['roofline']; u=d['reservoir_only']['roofline_unpaced']
print('$v', d['value'], d['ms_per_step'], 'upd beside', r['update_avg_ms'], 'upd alone', u['update_avg_ms'], 'res-only', d['reservoir_only']['value'])"
  done
done
