# r05w: the bench over step counts / warmups (what the driver's 20-step command loses)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; o=gpurun_out/r05w; mkdir -p $o
for cfg in "--steps 20 --warmup 5" "--steps 20 --warmup 5" "--steps 20 --warmup 50" "--steps 100 --warmup 5" "--steps 300 --warmup 20"; do
  f=$o/$(echo $cfg | tr -d ' -')
  SML_BENCH_HOST=1 timeout -k 10 300 python -u bench.py $cfg --no-cpu-baseline --train-regions 0 --speedy-steps 0 --reservoir-steps 0 > $f.json 2> $f.err || { tail $f.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); print('$cfg', d['value'], d['ms_per_step'], (d.get('run_speedy_poll') or {}).get('value_without_poll'))"
  grep "host:" $f.err | head -2
done
