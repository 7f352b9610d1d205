#!/bin/bash
# SPEEDY window counters (tools/speedy_pmc.py): one kernel trace, one counter pass.
set -euo pipefail
R=${1:-r02}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/speedy_pmc_$R
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES \
    SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_BUSY_CU_CYCLES \
    GRBM_GUI_ACTIVE -d "$OUT/pmc" -o pmc --output-format csv -- python3 "$ROOT/tools/speedy_pmc.py" run 3 \
    > "$OUT/run.log" 2>&1
python3 "$ROOT/tools/speedy_pmc.py" summarize "$OUT" "$R" > "$OUT/summary.json"
