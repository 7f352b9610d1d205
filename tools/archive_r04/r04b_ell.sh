#!/bin/bash
# r04b: the ELL layout change -- its parity tests, then a same-box A/B of the update
set -o pipefail
mkdir -p gpurun_out/r04b
T="timeout -k 10"
$T 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_reservoir_gpu.py \
  -k "ell_layouts or balanced or long_rows or f64_storage or fused_begin or predict_small" \
  > gpurun_out/r04b/tests.log 2>&1 || { tail -30 gpurun_out/r04b/tests.log; exit 1; }
tail -3 gpurun_out/r04b/tests.log
B="python -u bench.py --no-cpu-baseline --train-regions 0 --speedy-steps 0"
for i in 1 2; do
  for v in A B; do
    if [ $v = A ]; then export SML_LIB=$PWD/ablib/libspeedyml_head.so; else unset SML_LIB; fi
    $T 240 $B > gpurun_out/r04b/ab_$v$i.json 2> gpurun_out/r04b/ab_$v$i.err || { tail -5 gpurun_out/r04b/ab_$v$i.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/r04b/ab_$v$i.json')); r=d['roofline']; u=d['reservoir_only']['roofline_unpaced']
print('$v', d['value'], d['ms_per_step'], 'upd beside', r['update_avg_ms'], 'upd alone', u['update_avg_ms'], 'res-only', d['reservoir_only']['value'])"
  done
done
