#!/bin/bash
# r04k: the window's write-through hand-offs (SML_DYN_WT=1, the template form) vs the
# default write-back stores -- same-box A/B, N = 1 and the window alone
set -o pipefail
mkdir -p gpurun_out/r04k
T="timeout -k 10"
B="python -u bench.py --no-cpu-baseline --train-regions 0 --reservoir-steps 0"
for i in 1 2; do
  for v in A B; do
    unset SML_DYN_WT; [ $v = B ] && export SML_DYN_WT=1
    $T 300 $B > gpurun_out/r04k/w_$v$i.json 2> gpurun_out/r04k/w_$v$i.err || { tail -5 gpurun_out/r04k/w_$v$i.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/r04k/w_$v$i.json').read().strip().splitlines()[-1]); s=d['speedy_step']; r=s['roofline']
print('$v', d['value'], d['ms_per_step'], 'window', s['window_ms_graph_physics'], 'gs', r['k_st_gridspec']['span_us'], r['k_st_gridspec']['phases_us'], 'spec', r['k_st_spec']['span_us'], r['k_st_spec']['phases_us'])"
  done
done
