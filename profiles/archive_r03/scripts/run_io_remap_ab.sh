#!/bin/bash
# r03g: iogrid's FFT kernels (run_model's entry specx and exit gridx, on the hybrid
# step's critical path) with the four variables of one (level, latitude) on
# neighbouring transforms (coalesced (var, x, y, z) grid access); parity first, then a
# same-box A/B against HEAD (ab/HEAD) and one traced pass each
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/io
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_spectral_gpu.py tests/test_run_model_gpu.py tests/test_hybrid_gpu.py tests/test_fortran_hybrid_gpu.py > gpurun_out/io/tests.log 2>&1
rc=$?; tail -1 gpurun_out/io/tests.log; [ $rc -eq 0 ] || exit $rc
HEADLIB=$GRAFT_REPO_ROOT/ab/HEAD/speedy-ml-1_amd/lib/libspeedyml.so
B="python -u bench.py --no-cpu-baseline --train-regions 0 --speedy-steps 0 --reservoir-steps 0"
for i in 1 2 3; do
  for e in "SML_LIB=$HEADLIB" "X=0"; do
    env $e timeout -k 10 200 $B > gpurun_out/io/b.json 2> gpurun_out/io/b.err || { tail -5 gpurun_out/io/b.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/io/b.json').read().strip().splitlines()[-1]); print('${e##*/} rep $i', d['value'], d['ms_per_step'])"
  done
done
cd /tmp && export TMPDIR=/tmp
for e in "SML_LIB=$HEADLIB" "X=0"; do
  n=$(echo "${e##*/}" | tr -c 'A-Za-z0-9\n' '_')
  env $e timeout -k 10 300 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/io/$n" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 40 --warmup 5 --no-cpu-baseline --train-regions 0 --speedy-steps 0 --reservoir-steps 0 > "$GRAFT_REPO_ROOT/gpurun_out/io/$n.log" 2>&1 || { tail -5 "$GRAFT_REPO_ROOT/gpurun_out/io/$n.log"; exit 1; }
done
echo traced ok
