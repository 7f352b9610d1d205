#!/bin/bash
# r03g: does the host keep ahead of the GPU (SML_BENCH_HOST=1: enqueue time per step),
# and do more hardware queues per process change the overlapped loop (GPU_MAX_HW_QUEUES=8)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/hq
B="python -u bench.py --no-cpu-baseline --train-regions 0 --speedy-steps 0 --reservoir-steps 0"
SML_BENCH_HOST=1 timeout -k 10 200 $B > gpurun_out/hq/b.json 2> gpurun_out/hq/host.err || { tail -5 gpurun_out/hq/host.err; exit 1; }
grep "host:" gpurun_out/hq/host.err
for i in 1 2 3; do
  for e in "X=0" "GPU_MAX_HW_QUEUES=8"; do
    env $e timeout -k 10 200 $B > gpurun_out/hq/b.json 2> gpurun_out/hq/b.err || { tail -5 gpurun_out/hq/b.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/hq/b.json').read().strip().splitlines()[-1]); print('$e rep $i', d['value'], d['ms_per_step'])"
  done
done
