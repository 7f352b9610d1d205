#!/bin/bash
# r03 rocprofv3 evidence for the default 1-GPU bench (slab ocean on):
#   1. kernel trace + stats, 2. FETCH_SIZE pass, 3. WRITE_SIZE pass, 4. the SPEEDY
#   window's counter pass (tools/speedy_pmc.py); summaries into profiles/ by
#   profiles/summarize.py and tools/speedy_pmc.py.  The counter passes run the loop with
#   SML_HOP_AUTO: rocprofv3 --pmc sets ROCPROF_COUNTER_COLLECTION and the loop takes
#   event hops by itself (checked first by tools/hop_mode_check.py, which steps only
#   when the effective mode is events).
set -euo pipefail
R=${1:-r03}
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
OUT=$ROOT/gpurun_out/prof_$R
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
unset SML_HYBRID_EVENTS
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES -d "$OUT/hopcheck" -o hop --output-format csv \
    -- python3 "$ROOT/tools/hop_mode_check.py" > "$OUT/hopcheck.log" 2>&1
grep -q "effective events" "$OUT/hopcheck.log" || { echo "hop mode not events under --pmc"; cat "$OUT/hopcheck.log"; exit 1; }
ARGS="$ROOT/bench.py --steps 20 --warmup 3 --no-cpu-baseline --train-regions 0 --speedy-steps 8 --reservoir-steps 10"
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o trace --output-format csv \
    -- python3 $ARGS > "$OUT/trace_bench.json" 2> "$OUT/trace_bench.err"
timeout -k 10 500 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o fetch --output-format csv \
    -- python3 $ARGS > "$OUT/fetch_bench.json" 2> "$OUT/fetch_bench.err"
timeout -k 10 500 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o write --output-format csv \
    -- python3 $ARGS > "$OUT/write_bench.json" 2> "$OUT/write_bench.err"
python3 "$ROOT/profiles/summarize.py" "$OUT" "$R"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES \
    SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 \
    SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE -d "$OUT/speedy" -o pmc --output-format csv \
    -- python3 "$ROOT/tools/speedy_pmc.py" run > "$OUT/speedy_run.log" 2>&1
python3 "$ROOT/tools/speedy_pmc.py" summarize "$OUT/speedy" "$R"
echo "collect $R ok"
