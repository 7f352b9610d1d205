# r03d: shortwave split across the row block's waves (tree), + fband in LDS (ab/fbl),
# vs the last commit (ab/head): tests on tree and fbl, sw-step phases, headline A/B x2
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
lib() { [ "$1" = tree ] && echo "" || echo "$GRAFT_REPO_ROOT/ab/$1/speedy-ml-1_amd/lib/libspeedyml.so"; }
for v in tree fbl; do
  SML_LIB=$(lib $v) timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_physics_gpu.py tests/test_window_ref_gpu.py tests/test_dynamics_gpu.py tests/test_run_model_gpu.py > gpurun_out/sw3_tests_$v.log 2>&1
  rc=$?; echo "tests $v: $(tail -1 gpurun_out/sw3_tests_$v.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/sw3_tests_$v.log; exit $rc; }
done
for v in head tree fbl; do
  for n in 22 24; do
    SML_LIB=$(lib $v) NLEAP=$n timeout -k 10 200 python -u tools/probe_phase_contention.py > gpurun_out/sw3_$v$n.log 2>&1 || { tail -5 gpurun_out/sw3_$v$n.log; exit 1; }
    echo "== $v NLEAP=$n"; grep -E "window alone|physics|gridx|grid.span" gpurun_out/sw3_$v$n.log
  done
done
for i in 1 2; do
  for v in head tree fbl; do
    SML_LIB=$(lib $v) timeout -k 10 200 python -u bench.py --no-cpu-baseline --train-regions 0 --reservoir-steps 0 > gpurun_out/sw3_$v$i.json 2> gpurun_out/sw3_$v$i.err || { tail -5 gpurun_out/sw3_$v$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/sw3_$v$i.json')); print('$v', d['value'], d['ms_per_step'], 'window', d['speedy_step']['window_ms_graph_physics'])"
  done
done
