# r05q: the quad physics row kernel -- bitwise / parity tests, then a same-box A/B
# of the default bench with SML_DYN_QUAD=0 (one lane per column) and 1 (quads)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; o=gpurun_out/r05q; mkdir -p $o
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_physics_gpu.py \
  tests/test_window_ref_gpu.py > $o/tests.log 2>&1 || { tail -40 $o/tests.log; exit 1; }
grep -E "passed|failed" $o/tests.log | tail -2
for rep in 1 2; do
  for q in 0 1; do
    f=$o/q${q}_$rep
    SML_DYN_QUAD=$q timeout -k 10 300 python -u bench.py --no-cpu-baseline --train-regions 0 > $f.json 2> $f.err || { tail $f.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); s=d.get('speedy_step') or {}
r=(s.get('roofline') or {}).get('k_st_gridspec') or {}
print('quad $q rep $rep', d['value'], d['ms_per_step'], 'window', s.get('window_ms_graph_physics'), 'gs', r.get('span_us'), r.get('phases_us'))"
  done
done
