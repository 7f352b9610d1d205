# round 4: the window as a replayed graph (default) vs direct launches, same box
set -o pipefail
mkdir -p gpurun_out
B="--no-cpu-baseline --train-regions 0 --speedy-steps 0 --reservoir-steps 0"
run() { name=$1; shift; echo "== $name" >> gpurun_out/bench7.err; timeout -k 10 180 "$@" > gpurun_out/$name.json 2>> gpurun_out/bench7.err || exit 3; }
run h_graph python bench.py $B
run h_nograph env SML_DYN_NOGRAPH=1 python bench.py $B
run h_graph2 python bench.py $B
run h_nograph2 env SML_DYN_NOGRAPH=1 python bench.py $B
run h_sim8_graph python bench.py $B --sim-ranks 8
run h_sim8_nograph env SML_DYN_NOGRAPH=1 python bench.py $B --sim-ranks 8
