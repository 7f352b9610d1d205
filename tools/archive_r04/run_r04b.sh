# round 4: the sharded slab test after the fix, then traced --sim-ranks 8 steps in both
# chain modes (kernel order on the streams around the window), and same-box A/Bs of
# the interleaved vp_sum (one-pass readout, reservoir-only leg)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_sharded_gpu.py tests/test_reservoir_gpu.py tests/test_hybrid_gpu.py > gpurun_out/t2.log 2>&1
echo "pytest rc $?" >> gpurun_out/t2.log
export TMPDIR=/tmp
ROOT=$PWD
B="--no-cpu-baseline --train-regions 0 --speedy-steps 0"
for mode in speedy two-streams; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $ROOT/gpurun_out/tr_$mode -o tr --output-format csv -- python3 $ROOT/bench.py $B --reservoir-steps 0 --sim-ranks 8 --chain $mode --steps 12 --warmup 3 > $ROOT/gpurun_out/tr_$mode.json 2>> $ROOT/gpurun_out/bench2.err) || exit 2
done
run() { name=$1; shift; echo "== $name" >> gpurun_out/bench2.err; timeout -k 10 180 "$@" > gpurun_out/$name.json 2>> gpurun_out/bench2.err || exit 3; }
run c_default python bench.py $B
run c_default2 python bench.py $B
