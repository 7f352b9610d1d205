# paced readout: step time + HBM traffic of the v_ml readout (one FETCH_SIZE pass)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
WAVES="${WAVES:-2048}" bash profiles/run_readwaves.sh || exit $?
cd /tmp && timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $GRAFT_REPO_ROOT/gpurun_out/rdt -o f --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 8 --warmup 2 --no-cpu-baseline --train-regions 0 --speedy-steps 0 --reservoir-steps 4 > $GRAFT_REPO_ROOT/gpurun_out/rdt.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT && python3 - <<'PY'
import csv,glob,collections
f=glob.glob('gpurun_out/rdt/**/*counter_collection.csv',recursive=True)[0]
acc=collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    n=r['Kernel_Name']
    if 'k_res_readout' in n: acc[n[:45]].append(float(r['Counter_Value']))
for k,v in acc.items(): print(k, len(v), 'FETCH KiB/launch (raw)', sum(v)/len(v), '-> GB x2', 2*sum(v)/len(v)*1024/1e9)
PY
