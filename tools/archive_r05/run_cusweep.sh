# sweep of the overlapped hybrid step's knobs on one GPU (bench.py, short legs)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/cus
run() {  # run NAME ENV... -- bench args
  local name=$1; shift
  timeout -k 10 200 env "$@" python -u bench.py --no-cpu-baseline --train-regions 0 --reservoir-steps 0 --speedy-steps 0 --steps 50 > gpurun_out/cus/$name.json 2> gpurun_out/cus/$name.err || { tail gpurun_out/cus/$name.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/cus/$name.json').read().strip().splitlines()[-1]); print('$name', d['value'], d['ms_per_step'], d['roofline']['readout_avg_ms'])"
}
for w in 2048 0 1024 1536 3072 4096 2048; do run rw$w SML_READ_WAVES=$w; done
