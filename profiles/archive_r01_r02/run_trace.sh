# kernel trace + stats of the default-shaped hybrid bench (no counters): per-kernel durations
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=${R:-r02t}
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/trace_$R -o trace --output-format csv \
  -- python3 $GRAFT_REPO_ROOT/bench.py --steps 40 --warmup 5 --no-cpu-baseline --train-regions 0 --speedy-steps 0 --reservoir-steps 0 \
  > $GRAFT_REPO_ROOT/gpurun_out/trace_$R.json 2> $GRAFT_REPO_ROOT/gpurun_out/trace_$R.err || exit 1
f=$(find $GRAFT_REPO_ROOT/gpurun_out/trace_$R -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:30]:
    print(f"{r['Name'][:60]:60s} {r['Calls']:>6s} {float(r['AverageNs'])/1e3:9.2f} us {float(r['Percentage']):6.2f}%")
PY
