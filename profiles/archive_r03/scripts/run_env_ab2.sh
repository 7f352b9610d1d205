# r03d: reservoir CUs (SML_RES_CUS) and the fused begin (SML_BEGIN=1) at HEAD, same box
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for i in 1 2; do
  for e in "X=0" "SML_RES_CUS=176" "SML_RES_CUS=160" "SML_BEGIN=1"; do
    env $e timeout -k 10 200 python -u bench.py --no-cpu-baseline --train-regions 0 --speedy-steps 0 --reservoir-steps 0 > gpurun_out/env2.json 2> gpurun_out/env2.err || { tail -5 gpurun_out/env2.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/env2.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$e rep $i', d['value'], d['ms_per_step'], r['readout_avg_ms'], r['update_avg_ms'])"
  done
done
