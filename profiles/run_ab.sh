# same-box A/B of two library builds: A = $SML_LIB_A (tools/ab_build.sh REV), B = the
# tree's own build; the headline bench (no CPU leg, no training, speedy leg on),
# alternated N times
set -o pipefail
mkdir -p gpurun_out
N=${N:-3}
B="python -u bench.py --no-cpu-baseline --train-regions 0 --reservoir-steps 0"
for i in $(seq 1 $N); do
  for v in A B; do
    if [ $v = A ]; then export SML_LIB=$SML_LIB_A; else unset SML_LIB; fi
    timeout -k 10 200 $B > gpurun_out/ab_$v$i.json 2> gpurun_out/ab_$v$i.err || { tail -5 gpurun_out/ab_$v$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab_$v$i.json')); print('$v', d['value'], d['ms_per_step'], 'window', d['speedy_step']['window_ms_graph_physics'])"
  done
done
