# r03: library variants (ab/<name>/..., tools/ab_variant.sh; "tree" = the tree's build):
# the window tests on the tree's build, then per variant the phase-contention probe
# and the headline bench, alternated REPS times
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_physics_gpu.py tests/test_window_ref_gpu.py -x -q --timeout 240 --timeout-method thread > gpurun_out/var_tests.log 2>&1
rc=$?; tail -2 gpurun_out/var_tests.log; [ $rc -eq 0 ] || exit $rc
lib() { [ "$1" = tree ] && echo "" || echo "$GRAFT_REPO_ROOT/ab/$1/speedy-ml-1_amd/lib/libspeedyml.so"; }
for v in $VARIANTS; do
  SML_LIB=$(lib $v) timeout -k 10 200 python -u tools/probe_phase_contention.py > gpurun_out/var_pc_$v.log 2>&1 || { tail -5 gpurun_out/var_pc_$v.log; exit 1; }
  echo "$v $(grep 'window alone' gpurun_out/var_pc_$v.log) | $(grep -E 'grid.span|spec.span' gpurun_out/var_pc_$v.log | tr -s ' ' | tr '\n' ';')"
done
for i in $(seq 1 ${REPS:-2}); do
  for v in $VARIANTS; do
    SML_LIB=$(lib $v) timeout -k 10 200 python -u bench.py --no-cpu-baseline --train-regions 0 --reservoir-steps 0 > gpurun_out/var_$v$i.json 2> gpurun_out/var_$v$i.err || { tail -5 gpurun_out/var_$v$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/var_$v$i.json')); print('$v', d['value'], d['ms_per_step'], 'window', d['speedy_step']['window_ms_graph_physics'])"
  done
done
