# r05h: evidence at the pair-kernel default (tests, smoke, bench, driver command, rocprof),
# then the SPEEDY counter pass for the row kernel's work per dispatch (tools/speedy_pmc.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=r05h bash tools/gpu/evidence.sh || exit 1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
(cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES \
   SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE \
   -d $R/gpurun_out/pmc_r05h -o pmc --output-format csv -- python3 $R/tools/speedy_pmc.py run) > $R/gpurun_out/pmc_r05h.log 2>&1 || { tail $R/gpurun_out/pmc_r05h.log; exit 1; }
echo pmc ok
