#!/bin/bash
# r04e: the chain on SPEEDY's stream without hop kernels (the finish waits for its begin
# in-kernel, the entry specx signals the assembled grid) -- tests, then A (two streams)
# / B (SPEEDY's stream) at N = 1 and in the 8-rank share
set -o pipefail
mkdir -p gpurun_out/r04e
T="timeout -k 10"
$T 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_hybrid_gpu.py tests/test_sharded_gpu.py \
  > gpurun_out/r04e/tests.log 2>&1 || { tail -30 gpurun_out/r04e/tests.log; exit 1; }
tail -1 gpurun_out/r04e/tests.log
B="python -u bench.py --no-cpu-baseline --train-regions 0 --reservoir-steps 0 --speedy-steps 0"
for i in 1 2; do
  for v in A B; do
    C=two-streams; [ $v = B ] && C=speedy
    $T 240 $B --chain $C > gpurun_out/r04e/n1_$v$i.json 2> gpurun_out/r04e/n1_$v$i.err || { tail -5 gpurun_out/r04e/n1_$v$i.err; exit 1; }
    $T 240 $B --chain $C --sim-ranks 8 > gpurun_out/r04e/s8_$v$i.json 2> gpurun_out/r04e/s8_$v$i.err || { tail -5 gpurun_out/r04e/s8_$v$i.err; exit 1; }
    python3 -c "
import json; a=json.load(open('gpurun_out/r04e/n1_$v$i.json')); b=json.load(open('gpurun_out/r04e/s8_$v$i.json'))
print('$v', 'N1', a['value'], 'sim8', b['value'], b['ms_per_step'])"
  done
done
