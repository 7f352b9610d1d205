# per-kernel trace of the SPEEDY step, fused (default) and unfused (SML_DYN_UNFUSED=1)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
A="bench.py --steps 5 --warmup 2 --no-cpu-baseline --train-regions 0 --reservoir-steps 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/dynprof_fused -o run --output-format csv -- python3 $A > gpurun_out/dynprof_fused.log 2>&1 || exit $?
SML_DYN_UNFUSED=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/dynprof_unfused -o run --output-format csv -- python3 $A > gpurun_out/dynprof_unfused.log 2>&1 || exit $?
echo done
