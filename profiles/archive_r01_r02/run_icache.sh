# instruction-fetch counters of the SPEEDY step kernels (one kernel-trace + pmc pass each)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/icache; export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --list-avail > gpurun_out/icache/avail.txt 2>&1
grep -o "SQC_ICACHE[A-Z_]*\|SQ_IFETCH[A-Z_]*\|SQ_WAIT_INST[A-Z_]*\|SQ_INST_CYCLES[A-Z_]*\|SQ_WAVE_CYCLES\|SQ_BUSY_CYCLES\|SQ_WAIT_ANY\|SQC_TC_INST_REQ\|SQ_INSTS_VALU\b\|SQ_INSTS_LDS\|SQ_WAIT_INST_LDS" gpurun_out/icache/avail.txt | sort -u
cd /tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAVES SQ_INSTS_VALU -d $GRAFT_REPO_ROOT/gpurun_out/icache/p1 -o pmc --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/speedy_pmc.py run 2 > $GRAFT_REPO_ROOT/gpurun_out/icache/run1.log 2>&1
echo rc=$?
tail -3 $GRAFT_REPO_ROOT/gpurun_out/icache/run1.log
