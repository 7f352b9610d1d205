#!/bin/bash
# profiles/collect.sh ROUND -- rocprofv3 evidence for the default 1-GPU bench:
#   1. kernel trace + stats (per-kernel average durations)
#   2. FETCH_SIZE pass, 3. WRITE_SIZE pass (separate passes: TCC slots, MI355X_MICROARCH.md)
# Raw output goes to gpurun_out/prof_<ROUND>/; summarize.py condenses it into profiles/.
set -euo pipefail
R=${1:-r01}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/prof_$R
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
ARGS="$ROOT/bench.py --steps 20 --warmup 3 --no-cpu-baseline --train-regions 0 --speedy-steps 8 --reservoir-steps 10"
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o trace --output-format csv \
    -- python3 $ARGS > "$OUT/trace_bench.json" 2> "$OUT/trace_bench.err"
# counter passes serialise the dispatches, which deadlocks the loop's CP wait-value
# hops between its two streams: those passes take the event hops (SML_HYBRID_EVENTS=1;
# the per-kernel traffic is the same)
export SML_HYBRID_EVENTS=1
timeout -k 10 500 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o fetch --output-format csv \
    -- python3 $ARGS > "$OUT/fetch_bench.json" 2> "$OUT/fetch_bench.err"
timeout -k 10 500 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o write --output-format csv \
    -- python3 $ARGS > "$OUT/write_bench.json" 2> "$OUT/write_bench.err"
python3 "$ROOT/profiles/summarize.py" "$OUT" "$R"
