#!/bin/bash
# r04i: per-kernel times of the training leg (rocprofv3 kernel trace + stats)
set -o pipefail
mkdir -p gpurun_out/r04i
export TMPDIR=/tmp
R=$PWD
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r04i/trace" -o trace --output-format csv \
  -- python3 $R/bench.py --no-cpu-baseline --steps 1 --warmup 0 --reservoir-steps 0 --speedy-steps 0 \
  > "$R/gpurun_out/r04i/bench.json" 2> "$R/gpurun_out/r04i/bench.err" || { tail -5 "$R/gpurun_out/r04i/bench.err"; exit 1; }
f=$(ls $R/gpurun_out/r04i/trace/*/trace_kernel_stats.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(find $R/gpurun_out/r04i/trace -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:20]:
    print(f"{r['Name'][:70]:70s} {int(r['Calls']):6d} {float(r['TotalDurationNs'])/1e6:9.2f} ms {float(r['AverageNs'])/1e3:9.1f} us")
PY
