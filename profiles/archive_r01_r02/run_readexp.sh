set -e
A="--no-cpu-baseline --train-regions 0 --speedy-steps 0 --steps 30"
for w in 4 8 2; do
  SML_READ_WPB=$w timeout -k 10 200 python -u bench.py $A > gpurun_out/rd_$w.json 2>/dev/null
  python -c "import json;d=json.load(open('gpurun_out/rd_$w.json'));r=d['roofline'];ro=d['reservoir_only']['roofline_unpaced'];print('$w', d['value'], r['readout_avg_ms'], ro['readout_avg_ms'], ro['frac'])"
done
