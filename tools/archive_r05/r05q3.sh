# r05q3: quad physics stamps, the bitwise test, and a same-box A/B (SML_DYN_QUAD 0 / 1)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; o=gpurun_out/r05q; mkdir -p $o; tag=${1:-x}
SML_LIB=abx/pst/speedy-ml-1_amd/lib/libspeedyml.so timeout -k 10 200 python -u tools/probe_pstq.py > $o/pstq_$tag.txt 2>&1 || { tail $o/pstq_$tag.txt; exit 1; }
grep -v amdgpu.ids $o/pstq_$tag.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_physics_gpu.py -k quad > $o/t_$tag.log 2>&1 || { tail -30 $o/t_$tag.log; exit 1; }
tail -1 $o/t_$tag.log
for q in 0 1; do
  f=$o/ab_${tag}_q$q
  SML_DYN_QUAD=$q timeout -k 10 300 python -u bench.py --no-cpu-baseline --train-regions 0 > $f.json 2> $f.err || { tail $f.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); s=d.get('speedy_step') or {}
r=(s.get('roofline') or {}).get('k_st_gridspec') or {}
print('quad $q', d['value'], d['ms_per_step'], 'window', s.get('window_ms_graph_physics'), 'gs', r.get('span_us'), r.get('phases_us'))"
done
