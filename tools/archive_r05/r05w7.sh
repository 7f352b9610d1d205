# r05w7: the third pair wave on wave 7 (SIMD 3, beside the half-full moist wave) vs wave 6 -- same box; bitwise check
set -o pipefail
cd "$GRAFT_REPO_ROOT"; o=gpurun_out/r05w7; mkdir -p $o
SML_LIB=abx/w7/speedy-ml-1_amd/lib/libspeedyml.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_physics_gpu.py -k "bitwise" > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
true
for rep in 3 4 5; do
  for q in head w7; do
    f=$o/${q}_$rep
    if [ $q = w7 ]; then export SML_LIB=abx/w7/speedy-ml-1_amd/lib/libspeedyml.so; else unset SML_LIB; fi
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --train-regions 0 > $f.json 2> $f.err || { tail $f.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); s=d.get('speedy_step') or {}
r=(s.get('roofline') or {}).get('k_st_gridspec') or {}
print('$q rep $rep', d['value'], d['ms_per_step'], 'window', s.get('window_ms_graph_physics'), 'gs', r.get('span_us'), r.get('phases_us'))"
  done
done
