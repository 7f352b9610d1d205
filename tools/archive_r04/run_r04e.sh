# round 4: the expm1 tanh in the state update
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_reservoir_gpu.py tests/test_hybrid_gpu.py tests/test_full_size_gpu.py tests/test_slab_gpu.py > gpurun_out/t5.log 2>&1
echo "pytest rc $?" >> gpurun_out/t5.log
B="--no-cpu-baseline --train-regions 0 --speedy-steps 0"
run() { name=$1; shift; echo "== $name" >> gpurun_out/bench5.err; timeout -k 10 180 "$@" > gpurun_out/$name.json 2>> gpurun_out/bench5.err || exit 3; }
run f_1 python bench.py $B
run f_2 python bench.py $B
