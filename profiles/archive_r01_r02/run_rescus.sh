set -e
A="--no-cpu-baseline --train-regions 0 --reservoir-steps 0 --speedy-steps 0 --steps 60"
for cfg in 192 128 160 192 128 160; do
  SML_RES_CUS=$cfg timeout -k 10 200 python -u bench.py $A > gpurun_out/rc_$cfg.json 2>/dev/null
  python -c "import json;d=json.load(open('gpurun_out/rc_$cfg.json'));r=d['roofline'];print('$cfg', d['value'], d['ms_per_step'], r['readout_avg_ms'])"
done
