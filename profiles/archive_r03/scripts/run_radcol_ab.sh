# r03d: the radiation state in registers on shortwave steps (tree) vs HEAD (ab/head):
# physics / window / hybrid tests, the shortwave-step phases, headline A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_physics_gpu.py tests/test_window_ref_gpu.py tests/test_dynamics_gpu.py tests/test_run_model_gpu.py tests/test_hybrid_gpu.py > gpurun_out/rc_tests.log 2>&1
rc=$?; tail -1 gpurun_out/rc_tests.log; [ $rc -eq 0 ] || { tail -30 gpurun_out/rc_tests.log; exit $rc; }
lib() { [ "$1" = tree ] && echo "" || echo "$GRAFT_REPO_ROOT/ab/$1/speedy-ml-1_amd/lib/libspeedyml.so"; }
for v in head tree; do
  SML_LIB=$(lib $v) NLEAP=22 timeout -k 10 200 python -u tools/probe_phase_contention.py > gpurun_out/rc_sw_$v.log 2>&1 || { tail -5 gpurun_out/rc_sw_$v.log; exit 1; }
  echo "== $v (last step shortwave)"; grep -E "window alone|physics|grid.span" gpurun_out/rc_sw_$v.log
done
for i in 1 2; do
  for v in head tree; do
    SML_LIB=$(lib $v) timeout -k 10 200 python -u bench.py --no-cpu-baseline --train-regions 0 --reservoir-steps 0 > gpurun_out/rc_$v$i.json 2> gpurun_out/rc_$v$i.err || { tail -5 gpurun_out/rc_$v$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/rc_$v$i.json')); print('$v', d['value'], d['ms_per_step'], 'window', d['speedy_step']['window_ms_graph_physics'])"
  done
done
