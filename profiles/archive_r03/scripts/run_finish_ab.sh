#!/bin/bash
# r03g: the v_p finish on the hybrid step's critical path -- W_out(:, 1:ncs) read once
# after the begin (SML_WLM_TOUCH=1, the finish then reads the memory-side cache) and
# more column loads in flight per thread (SML_VP_UNROLL=24 / 44 vs 12); parity first,
# then same-box headline A/B and one traced pass per variant for the finish's duration
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/fin
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_hybrid_gpu.py tests/test_reservoir_gpu.py -k"
K="overlapped or native_comm or pipelined or finish_assemble or sequential_chain"
SML_WLM_TOUCH=1 SML_VP_UNROLL=44 timeout -k 10 400 $T "$K" > gpurun_out/fin/tests44.log 2>&1
rc=$?; tail -1 gpurun_out/fin/tests44.log; [ $rc -eq 0 ] || exit $rc
SML_VP_UNROLL=24 timeout -k 10 400 $T "$K" > gpurun_out/fin/tests24.log 2>&1
rc=$?; tail -1 gpurun_out/fin/tests24.log; [ $rc -eq 0 ] || exit $rc
B="python -u bench.py --no-cpu-baseline --train-regions 0 --speedy-steps 0 --reservoir-steps 0"
for i in 1 2; do
  for e in "X=0" "SML_WLM_TOUCH=1" "SML_VP_UNROLL=24" "SML_VP_UNROLL=44" "SML_WLM_TOUCH=1 SML_VP_UNROLL=24"; do
    env $e timeout -k 10 200 $B > gpurun_out/fin/b.json 2> gpurun_out/fin/b.err || { tail -5 gpurun_out/fin/b.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/fin/b.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$e rep $i', d['value'], d['ms_per_step'], 'readout', r['readout_avg_ms'])"
  done
done
cd /tmp && export TMPDIR=/tmp
for e in "X=0" "SML_WLM_TOUCH=1" "SML_VP_UNROLL=24" "SML_VP_UNROLL=44"; do
  n=$(echo "$e" | tr -c 'A-Za-z0-9\n' '_')
  env $e timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/fin/$n" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 40 --warmup 5 --no-cpu-baseline --train-regions 0 --speedy-steps 0 --reservoir-steps 0 > "$GRAFT_REPO_ROOT/gpurun_out/fin/$n.log" 2>&1 || { tail -5 "$GRAFT_REPO_ROOT/gpurun_out/fin/$n.log"; exit 1; }
  f=$(find "$GRAFT_REPO_ROOT/gpurun_out/fin/$n" -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    if 'finish_grid' in r['Name'] or 'k_touch' in r['Name']: print('$e', r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,2), 'us')"
done
