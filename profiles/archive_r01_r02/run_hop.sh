# value hops vs event hops in the overlapped hybrid step, alternated (bench.py headline only)
set -o pipefail
mkdir -p gpurun_out
B="python -u bench.py --steps 300 --warmup 10 --no-cpu-baseline --train-regions 0 --reservoir-steps 0 --speedy-steps 0"
for i in 1 2 3 4; do
  timeout -k 10 200 $B > gpurun_out/hop_v$i.json 2> gpurun_out/hop_v$i.err || exit 1
  SML_HYBRID_EVENTS=1 timeout -k 10 200 $B > gpurun_out/hop_e$i.json 2> gpurun_out/hop_e$i.err || exit 1
done
for f in gpurun_out/hop_[ve]?.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'])"; done
