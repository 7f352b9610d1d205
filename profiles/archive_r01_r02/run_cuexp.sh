set -e
A="--no-cpu-baseline --train-regions 0 --reservoir-steps 0 --speedy-steps 0 --steps 40"
for cfg in "0 64" "8 64" "4 64" "2 64" "8 96" "0 96"; do
  set -- $cfg
  SML_SPEEDY_CU_STRIDE=$1 timeout -k 10 200 python -u bench.py $A --speedy-cus $2 > gpurun_out/cu_$1_$2.json 2>/dev/null
  python -c "import json;d=json.load(open('gpurun_out/cu_$1_$2.json'));print('$1 $2', d['value'], d['ms_per_step'])"
done
