# r03d: window variants (ab/<name>/..., "tree" = the tree's build): window parity tests
# on each, then the phase-contention probe per variant and the headline bench,
# alternated REPS times.  VARIANTS="tree prev s32"
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
lib() { [ "$1" = tree ] && echo "" || echo "$GRAFT_REPO_ROOT/ab/$1/speedy-ml-1_amd/lib/libspeedyml.so"; }
for v in $TESTED; do
  SML_LIB=$(lib $v) timeout -k 10 400 python -u -m pytest tests/test_window_ref_gpu.py tests/test_physics_gpu.py tests/test_dynamics_gpu.py -x -q --timeout 240 --timeout-method thread > gpurun_out/var_tests_$v.log 2>&1
  rc=$?; echo "tests $v: $(tail -1 gpurun_out/var_tests_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
for v in $VARIANTS; do
  SML_LIB=$(lib $v) timeout -k 10 200 python -u tools/probe_phase_contention.py > gpurun_out/var_pc_$v.log 2>&1 || { tail -5 gpurun_out/var_pc_$v.log; exit 1; }
  echo "== $v"; grep -E "window alone|span|load|gap" gpurun_out/var_pc_$v.log
done
for i in $(seq 1 ${REPS:-2}); do
  for v in $VARIANTS; do
    SML_LIB=$(lib $v) timeout -k 10 200 python -u bench.py --no-cpu-baseline --train-regions 0 --reservoir-steps 0 > gpurun_out/var_$v$i.json 2> gpurun_out/var_$v$i.err || { tail -5 gpurun_out/var_$v$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/var_$v$i.json')); print('$v', d['value'], d['ms_per_step'], 'window', d['speedy_step']['window_ms_graph_physics'])"
  done
done
