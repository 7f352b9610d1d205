# round 4: the exit's counter hand-off (SML_CHK_FLAG) and the unguarded vp_sum:
# tests that exercise run_model / the loop, then same-box A/Bs
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_run_model_gpu.py tests/test_hybrid_gpu.py tests/test_sharded_gpu.py tests/test_slab_gpu.py tests/test_reservoir_gpu.py tests/test_full_size_gpu.py tests/test_fortran_hybrid_gpu.py > gpurun_out/t3.log 2>&1
echo "pytest rc $?" >> gpurun_out/t3.log
B="--no-cpu-baseline --train-regions 0 --speedy-steps 0"
run() { name=$1; shift; echo "== $name" >> gpurun_out/bench3.err; timeout -k 10 180 "$@" > gpurun_out/$name.json 2>> gpurun_out/bench3.err || exit 3; }
run d_flag python bench.py $B
run d_event env SML_CHK_FLAG=0 python bench.py $B
run d_flag2 python bench.py $B
run d_event2 env SML_CHK_FLAG=0 python bench.py $B
run d_sim8_flag python bench.py $B --reservoir-steps 0 --sim-ranks 8
run d_sim8_event env SML_CHK_FLAG=0 python bench.py $B --reservoir-steps 0 --sim-ranks 8
