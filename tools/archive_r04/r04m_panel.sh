#!/bin/bash
# r04m: the Cholesky panel width (SML_CHOL_PANEL) with the padding skips -- solve time
set -o pipefail
mkdir -p gpurun_out/r04m
T="timeout -k 10"
B="python -u bench.py --no-cpu-baseline --steps 2 --warmup 1 --reservoir-steps 0 --speedy-steps 0"
for P in 8 4 6 12 16 8; do
  SML_CHOL_PANEL=$P $T 300 $B > gpurun_out/r04m/p$P.json 2> gpurun_out/r04m/p$P.err || { tail -5 gpurun_out/r04m/p$P.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r04m/p$P.json').read().strip().splitlines()[-1]); t=d['training']
print('panel $P', 'gram_ms', t['gram_ms'], 'solve_ms', t['solve_ms'], t['solve_roofline']['achieved'], t['solve_roofline']['frac'], 'ok', t['solve_info_ok'])"
done
