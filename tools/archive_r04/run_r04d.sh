# round 4: the batched vp_sum (the one-pass readout of the reservoir-only leg)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_reservoir_gpu.py tests/test_hybrid_gpu.py tests/test_full_size_gpu.py > gpurun_out/t4.log 2>&1
echo "pytest rc $?" >> gpurun_out/t4.log
B="--no-cpu-baseline --train-regions 0 --speedy-steps 0"
run() { name=$1; shift; echo "== $name" >> gpurun_out/bench4.err; timeout -k 10 180 "$@" > gpurun_out/$name.json 2>> gpurun_out/bench4.err || exit 3; }
run e_1 python bench.py $B
run e_2 python bench.py $B
