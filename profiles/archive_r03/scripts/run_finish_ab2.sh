#!/bin/bash
# r03g: the v_p finish with its per-output operands (v_ml, the unstandardize slot, its
# mean / std, the grid point) loaded with the gather's first index loads instead of
# after the sum; parity first, then a same-box A/B against HEAD (ab/HEAD) and one
# traced pass each for the finish's duration (SML_VP_UNROLL 12 / 24 beside it)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/fin2
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_hybrid_gpu.py tests/test_reservoir_gpu.py tests/test_slab_gpu.py tests/test_sharded_gpu.py > gpurun_out/fin2/tests.log 2>&1
rc=$?; tail -1 gpurun_out/fin2/tests.log; [ $rc -eq 0 ] || exit $rc
HEADLIB=$GRAFT_REPO_ROOT/ab/HEAD/speedy-ml-1_amd/lib/libspeedyml.so
B="python -u bench.py --no-cpu-baseline --train-regions 0 --speedy-steps 0 --reservoir-steps 0"
for i in 1 2 3; do
  for e in "SML_LIB=$HEADLIB" "X=0" "SML_VP_UNROLL=24"; do
    env $e timeout -k 10 200 $B > gpurun_out/fin2/b.json 2> gpurun_out/fin2/b.err || { tail -5 gpurun_out/fin2/b.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/fin2/b.json').read().strip().splitlines()[-1]); print('${e##*/} rep $i', d['value'], d['ms_per_step'])"
  done
done
cd /tmp && export TMPDIR=/tmp
for e in "SML_LIB=$HEADLIB" "X=0" "SML_VP_UNROLL=24"; do
  n=$(echo "${e##*/}" | tr -c 'A-Za-z0-9\n' '_')
  env $e timeout -k 10 300 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/fin2/$n" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 40 --warmup 5 --no-cpu-baseline --train-regions 0 --speedy-steps 0 --reservoir-steps 0 > "$GRAFT_REPO_ROOT/gpurun_out/fin2/$n.log" 2>&1 || { tail -5 "$GRAFT_REPO_ROOT/gpurun_out/fin2/$n.log"; exit 1; }
done
echo traced ok
