# kernel trace of the fused step (SML_DYN_FUSED=1)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
SML_DYN_FUSED=${FZ:-1} timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fprof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --train-regions 0 --reservoir-steps 0 --speedy-steps 8 > gpurun_out/fprof.log 2>&1 || exit $?
python3 - <<'PY'
import csv
r=list(csv.DictReader(open('gpurun_out/fprof/run_kernel_stats.csv')))
for x in r[:20]:
    print(f"{x['Name'][:60]:60s} {int(x['Calls']):6d} {float(x['AverageNs'])/1000:8.2f} {float(x['TotalDurationNs'])/1e6:8.2f}")
PY
