set -e
A="--no-cpu-baseline --train-regions 0 --reservoir-steps 0 --speedy-steps 0 --steps 40"
for cfg in "64 192" "64 128" "64 160" "48 208" "64 96"; do
  set -- $cfg
  SML_RES_CUS=$2 timeout -k 10 200 python -u bench.py $A --speedy-cus $1 > gpurun_out/cu2_$1_$2.json 2>/dev/null
  python -c "import json;d=json.load(open('gpurun_out/cu2_$1_$2.json'));r=d['roofline'];print('$1 $2', d['value'], d['ms_per_step'], r['readout_avg_ms'], r['update_avg_ms'])"
done
