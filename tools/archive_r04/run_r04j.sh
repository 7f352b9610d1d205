# round 4: --sim-ranks with the other ranks' rows filled once (the entry check passes, the exit integrates)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="--no-cpu-baseline --train-regions 0 --speedy-steps 0 --reservoir-steps 0"
timeout -k 10 240 rocprofv3 --kernel-trace -d gpurun_out/tr_sim8f -o tr -- python3 bench.py $B --steps 20 --warmup 3 --sim-ranks 8 > gpurun_out/tr_sim8f.json 2> gpurun_out/tr_sim8f.err || exit 3
for n in 2 4 8; do timeout -k 10 180 python3 bench.py $B --sim-ranks $n > gpurun_out/b_sim${n}f.json 2>> gpurun_out/b_j.err || exit 3; done
timeout -k 10 180 python3 bench.py $B > gpurun_out/b_n1f.json 2>> gpurun_out/b_j.err || exit 3
