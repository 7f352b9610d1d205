# round 4: state read by the readout in place (no x_aug copy) + kernel hops (SML_HYBRID_HOPK=1):
# the full GPU suite (default hops), the hybrid/slab tests under kernel hops, then a same-box A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests > gpurun_out/k_suite.log 2>&1 || exit 3
SML_HYBRID_HOPK=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_hybrid_gpu.py tests/test_slab_gpu.py tests/test_sharded_gpu.py > gpurun_out/k_tests.log 2>&1 || exit 3
B="--no-cpu-baseline --train-regions 0 --speedy-steps 0 --reservoir-steps 0"
run() { name=$1; shift; echo "== $name" >> gpurun_out/bench_k.err; timeout -k 10 180 "$@" > gpurun_out/$name.json 2>> gpurun_out/bench_k.err || exit 3; }
run k_wv1 python bench.py $B
run k_hk1 env SML_HYBRID_HOPK=1 python bench.py $B
run k_wv2 python bench.py $B
run k_hk2 env SML_HYBRID_HOPK=1 python bench.py $B
run k_s8wv1 python bench.py $B --sim-ranks 8
run k_s8hk1 env SML_HYBRID_HOPK=1 python bench.py $B --sim-ranks 8
run k_s8wv2 python bench.py $B --sim-ranks 8
run k_s8hk2 env SML_HYBRID_HOPK=1 python bench.py $B --sim-ranks 8
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SML_HYBRID_HOPK=1 timeout -k 10 240 rocprofv3 --kernel-trace -d gpurun_out/tr_s8hk -o tr -- python3 bench.py $B --steps 20 --warmup 3 --sim-ranks 8 > gpurun_out/tr_s8hk.json 2> gpurun_out/tr_s8hk.err || exit 3
