# MFMA-pipe counters of the training leg's kernels (16 regions), one --pmc pass each:
#   TAG=r06pm bash tools/gpu/pmc_train.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"; T=${TAG:-r06pm}; o=$GRAFT_REPO_ROOT/gpurun_out/$T; mkdir -p $o
export TMPDIR=/tmp
B="$GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --reservoir-steps 0 --speedy-steps 0 --steps 2 --warmup 1 --train-regions 16 ${TRAIN_ARGS:-}"
i=0
for pmc in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $pmc -d $o/p$i -o run --output-format csv -- python3 -u $B) > $o/p$i.out 2> $o/p$i.err || { tail -5 $o/p$i.err; exit 1; }
done
python3 - $o <<'PY'
import csv, sys, glob, collections
o = sys.argv[1]
for f in sorted(glob.glob(o + '/p*/**/*counter_collection.csv', recursive=True)):
    acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name']
        if not any(x in k for x in ('k_train', 'k_chol_update', 'k_chol_upanel', 'k_solve')): continue
        k = k.split('(')[0].split('::')[-1]
        acc[k][r['Counter_Name']] += float(r['Counter_Value'])
        n[(k, r['Counter_Name'])] += 1
    print(f)
    for k, d in acc.items():
        print('  ', k, {c: f"{v:.4g}" for c, v in d.items()})
PY
