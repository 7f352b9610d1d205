grep -E "PASSED|FAILED|ERROR" gpurun_out/t1.log | grep -v PASSED | head -20; tail -3 gpurun_out/t1.log; tail -2 gpurun_out/smoke.log
for f in gpurun_out/b_*.json; do echo -n "$f "; python -c "
import json,sys
try:
    d=json.loads(open('$f').read().strip().splitlines()[-1])
except Exception as e:
    print('no json', e); sys.exit(0)
r=d['roofline']; ro=d.get('reservoir_only') or {}
print(d['value'], d['ms_per_step'], 'upd', r['update_avg_ms'], 'rd', r['readout_avg_ms'], 'resonly', ro.get('value'), (ro.get('roofline_unpaced') or {}).get('update_avg_ms'), 'poll', (d.get('run_speedy_poll') or {}).get('cost_pct'))"; done
