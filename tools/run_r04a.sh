set -o pipefail
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_force_exchange_gpu.py tests/test_hybrid_gpu.py tests/test_sharded_gpu.py > gpurun_out/t1.log 2>&1 || exit 1
B="--no-cpu-baseline --train-regions 0 --reservoir-steps 0 --speedy-steps 0"
timeout -k 10 180 python bench.py $B > gpurun_out/b1.json 2> gpurun_out/b1.err || exit 2
timeout -k 10 180 python bench.py $B --sim-ranks 8 --chain speedy > gpurun_out/b_sim8_speedy.json 2>> gpurun_out/b1.err || exit 3
timeout -k 10 180 python bench.py $B --sim-ranks 8 --chain two-streams > gpurun_out/b_sim8_two.json 2>> gpurun_out/b1.err || exit 4
timeout -k 10 180 python bench.py $B --sim-ranks 8 --chain speedy > gpurun_out/b_sim8_speedy2.json 2>> gpurun_out/b1.err || exit 5
