# round 4: balanced update with fixed row buffers (no copy of in-flight loads), scalar row-table
# reads and unconditional row loads -- the reservoir tests, then depth 2 vs 3 beside the old build
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_reservoir_gpu.py > gpurun_out/m_tests.log 2>&1 || exit 3
SML_UPD_DEPTH=3 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_reservoir_gpu.py -k "balanced or bal" > gpurun_out/m_tests3.log 2>&1 || exit 3
B="--no-cpu-baseline --train-regions 0 --speedy-steps 0 --reservoir-steps 20"
run() { name=$1; shift; echo "== $name" >> gpurun_out/bench_m.err; timeout -k 10 180 "$@" > gpurun_out/$name.json 2>> gpurun_out/bench_m.err || exit 3; }
for rep in 1 2; do
run m_d2_$rep python bench.py $B
run m_d3_$rep env SML_UPD_DEPTH=3 python bench.py $B
done
