#!/bin/bash
# the step accounting (tools/probe_step_accounting.py) with the timeline build, then the
# default bench and its 8-rank share (--sim-ranks 8) for the same box
# usage: TAG=r06c bash tools/gpu/accounting.sh   (after: bash tools/build_variant.sh tl 'EXTRA=-DSML_TL')
set -o pipefail
cd "$GRAFT_REPO_ROOT"
T=${TAG:-r06c}
mkdir -p gpurun_out
SML_LIB=$GRAFT_REPO_ROOT/abx/tl/speedy-ml-1_amd/lib/libspeedyml.so timeout -k 10 300 python -u tools/probe_step_accounting.py \
    --json gpurun_out/${T}_accounting.json > gpurun_out/${T}_accounting.txt 2>&1 || { tail -20 gpurun_out/${T}_accounting.txt; exit 1; }
cat gpurun_out/${T}_accounting.txt
SML_LIB=$GRAFT_REPO_ROOT/abx/tl/speedy-ml-1_amd/lib/libspeedyml.so timeout -k 10 300 python -u tools/probe_step_accounting.py \
    --sim-ranks 8 --json gpurun_out/${T}_accounting_sim8.json > gpurun_out/${T}_accounting_sim8.txt 2>&1 || { tail -20 gpurun_out/${T}_accounting_sim8.txt; exit 1; }
cat gpurun_out/${T}_accounting_sim8.txt
[ "${BENCH:-1}" = 1 ] || exit 0
B="--no-cpu-baseline --train-regions 0 --reservoir-steps 0 --speedy-steps 0"
timeout -k 10 300 python -u bench.py $B > gpurun_out/${T}_n1.json 2> gpurun_out/${T}_n1.err || exit 1
timeout -k 10 300 python -u bench.py $B --sim-ranks 8 > gpurun_out/${T}_sim8.json 2> gpurun_out/${T}_sim8.err || exit 1
python3 -c "
import json
for n in ('n1', 'sim8'):
    d = json.loads(open('gpurun_out/${T}_' + n + '.json').read().strip().splitlines()[-1])
    print(n, d['value'], d['ms_per_step'])"
