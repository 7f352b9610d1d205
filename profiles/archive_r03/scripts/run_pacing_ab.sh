# r03d: the v_ml readout paced beside the window (SML_READ_WAVES caps its waves;
# 0 = one wave per item, the hybrid loop's default): same-box A/B of the headline
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for i in 1 2; do
  for w in 0 1280 1024 768; do
    SML_READ_WAVES=$w timeout -k 10 200 python -u bench.py --no-cpu-baseline --train-regions 0 --speedy-steps 0 --reservoir-steps 0 > gpurun_out/pace_$w$i.json 2> gpurun_out/pace_$w$i.err || { tail -5 gpurun_out/pace_$w$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/pace_$w$i.json').read().strip().splitlines()[-1]); r=d['roofline']; print('READ_WAVES=$w rep $i', d['value'], d['ms_per_step'], 'readout', r['readout_avg_ms'], 'update', r['update_avg_ms'])"
  done
done
