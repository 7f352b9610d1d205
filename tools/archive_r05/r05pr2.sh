# r05pr2: the pair kernel with the moist hand-over on shortwave steps: tests, A/B, stamps
set -o pipefail
cd "$GRAFT_REPO_ROOT"; o=gpurun_out/r05pr2; mkdir -p $o
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_physics_gpu.py tests/test_window_ref_gpu.py > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
SML_LIB=abx/pst/speedy-ml-1_amd/lib/libspeedyml.so timeout -k 10 200 python -u tools/probe_pstp.py 2>&1 | grep -v amdgpu.ids | tee $o/pstp.txt
for rep in 1 2; do
  for q in 0 2 e; do
    f=$o/q${q}_$rep
    if [ $q = e ]; then export SML_LIB=abx/early/speedy-ml-1_amd/lib/libspeedyml.so; else unset SML_LIB; fi
    SML_DYN_QUAD=${q/e/2} timeout -k 10 300 python -u bench.py --no-cpu-baseline --train-regions 0 > $f.json 2> $f.err || { tail $f.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); s=d.get('speedy_step') or {}
r=(s.get('roofline') or {}).get('k_st_gridspec') or {}
print('quad $q rep $rep', d['value'], d['ms_per_step'], 'window', s.get('window_ms_graph_physics'), 'gs', r.get('span_us'), r.get('phases_us'))"
  done
done
