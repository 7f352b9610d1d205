# round 4: sim8 with event hops vs wait-value hops (is the exit gridx slowed by the spinning wait?)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="--no-cpu-baseline --train-regions 0 --speedy-steps 0 --reservoir-steps 0 --steps 20 --warmup 3"
SML_HYBRID_EVENTS=1 timeout -k 10 240 rocprofv3 --kernel-trace -d gpurun_out/tr_sim8ev -o tr -- python3 bench.py $B --sim-ranks 8 > gpurun_out/tr_sim8ev.json 2> gpurun_out/tr_sim8ev.err || exit 3
B2="--no-cpu-baseline --train-regions 0 --speedy-steps 0 --reservoir-steps 0"
timeout -k 10 180 python3 bench.py $B2 --sim-ranks 8 > gpurun_out/b_sim8_wv.json 2>> gpurun_out/b_i.err || exit 3
SML_HYBRID_EVENTS=1 timeout -k 10 180 python3 bench.py $B2 --sim-ranks 8 > gpurun_out/b_sim8_ev.json 2>> gpurun_out/b_i.err || exit 3
