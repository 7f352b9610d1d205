# round 4: the full -m gpu suite (new: forced RCCL exchange, sharded slab + pipelined,
# restart, balanced update, grouped finish) and smoke(), then same-box bench A/Bs
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/t1.log 2>&1
rc=$?
echo "pytest rc $rc" >> gpurun_out/t1.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1   # test failures: still measure; a crash / timeout: stop
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 3
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
