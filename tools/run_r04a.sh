# round 4: new GPU tests (forced RCCL exchange, sharded slab + pipelined, restart,
# balanced update, grouped finish), then same-box bench A/Bs
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_reservoir_gpu.py tests/test_force_exchange_gpu.py tests/test_hybrid_gpu.py tests/test_sharded_gpu.py > gpurun_out/t1.log 2>&1 || exit 1
B="--no-cpu-baseline --train-regions 0 --speedy-steps 0"
run() { name=$1; shift; echo "== $name" >> gpurun_out/bench.err; timeout -k 10 180 "$@" > gpurun_out/$name.json 2>> gpurun_out/bench.err || exit 2; }
run b_default python bench.py $B
run b_old env SML_UPD_BAL=0 SML_FIN_UNGROUPED=1 python bench.py $B
run b_default2 python bench.py $B
run b_old2 env SML_UPD_BAL=0 SML_FIN_UNGROUPED=1 python bench.py $B
run b_sim8_speedy python bench.py $B --reservoir-steps 0 --sim-ranks 8 --chain speedy
run b_sim8_two python bench.py $B --reservoir-steps 0 --sim-ranks 8 --chain two-streams
run b_sim8_speedy2 python bench.py $B --reservoir-steps 0 --sim-ranks 8 --chain speedy
run b_sim8_two2 python bench.py $B --reservoir-steps 0 --sim-ranks 8 --chain two-streams
run b_n1_chain_speedy python bench.py $B --reservoir-steps 0 --chain speedy
run b_n1_chain_two python bench.py $B --reservoir-steps 0
