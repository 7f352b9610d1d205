# round 4: the reservoir's CU share at N = 1 with kernel hops (does a slower begin cost the window less?)
set -o pipefail
mkdir -p gpurun_out
B="--no-cpu-baseline --train-regions 0 --speedy-steps 0 --reservoir-steps 0"
run() { name=$1; shift; echo "== $name" >> gpurun_out/bench_l.err; timeout -k 10 180 "$@" > gpurun_out/$name.json 2>> gpurun_out/bench_l.err || exit 3; }
for rep in 1 2; do
run l_def$rep python bench.py $B
run l_c184_$rep env SML_RES_CUS=184 python bench.py $B
run l_c176_$rep env SML_RES_CUS=176 python bench.py $B
run l_c168_$rep env SML_RES_CUS=168 python bench.py $B
done
