# round 4: kernel traces of the N = 1 and the --sim-ranks 8 loop (current HEAD) for the chain timeline
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="--no-cpu-baseline --train-regions 0 --speedy-steps 0 --reservoir-steps 0 --steps 20 --warmup 3"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/tr_sim8 -o tr -- python3 bench.py $B --sim-ranks 8 > gpurun_out/tr_sim8.json 2> gpurun_out/tr_sim8.err || exit 3
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/tr_n1 -o tr -- python3 bench.py $B > gpurun_out/tr_n1.json 2> gpurun_out/tr_n1.err || exit 3
