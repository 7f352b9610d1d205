# end-of-round-2 evidence: SPEEDY counter pass (-> profiles/speedy_pmc.json, read by the
# bench), every GPU test, smoke(), the default bench line, rocprof collect, and the
# --sim-ranks diagnostic at N = 2 / 4 / 8
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
R=${R:-r02y}
bash profiles/run_speedy_pmc.sh $R && cp gpurun_out/speedy_pmc_$R/speedy_pmc.json profiles/speedy_pmc.json \
  && cp profiles/speedy_pmc.json gpurun_out/speedy_pmc_$R.json && echo "speedy pmc ok" || exit 1
R=$R bash profiles/run_r02.sh tests smoke bench prof || exit 1
for n in 2 4 8; do
  timeout -k 10 200 python -u bench.py --sim-ranks $n --no-cpu-baseline --train-regions 0 --reservoir-steps 0 --speedy-steps 0 > gpurun_out/${R}_sim$n.json 2> gpurun_out/${R}_sim$n.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/${R}_sim$n.json')); print('sim', $n, d['value'], d['ms_per_step'])"
done
