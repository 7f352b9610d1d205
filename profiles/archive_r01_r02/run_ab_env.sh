# same-box A/B of two environments for the tree's build: ENV_A vs ENV_B (e.g. ENV_B="SML_X=1"),
# the headline bench (no CPU leg, no training; the speedy leg on for the window time),
# alternated N times
set -o pipefail
mkdir -p gpurun_out
N=${N:-3}
B="python -u bench.py --no-cpu-baseline --train-regions 0 --reservoir-steps 0"
for i in $(seq 1 $N); do
  for v in A B; do
    if [ $v = A ]; then E="$ENV_A"; else E="$ENV_B"; fi
    env $E timeout -k 10 200 $B > gpurun_out/abe_$v$i.json 2> gpurun_out/abe_$v$i.err || { tail -5 gpurun_out/abe_$v$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/abe_$v$i.json')); print('$v', d['value'], d['ms_per_step'], 'window', d['speedy_step']['window_ms_graph_physics'], d['speedy_step']['roofline']['k_st_spec']['phases_us'])"
  done
done
