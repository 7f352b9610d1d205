# Kernel trace of the training leg under an env configuration:  bash tools/gpu/prof_train.sh <tag> "A=1 B=0"
set -o pipefail
cd "$GRAFT_REPO_ROOT"; tag=$1; o=$GRAFT_REPO_ROOT/gpurun_out/$tag; mkdir -p $o
export TMPDIR=/tmp
for kv in $2; do export $kv; done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof -o run --output-format csv -- python3 -u $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --reservoir-steps 0 --speedy-steps 0 --steps 2 --warmup 1) > $o/b.json 2> $o/b.err || { tail $o/b.err; exit 1; }
python3 - $o <<'PY'
import csv, sys, collections
o = sys.argv[1]
rows = list(csv.DictReader(open(o + '/prof/run_kernel_trace.csv')))
acc = collections.defaultdict(lambda: [0, 0.0])
for r in rows:
    n = r['Kernel_Name']
    if 'k_chol' in n or 'k_solve' in n or 'k_train' in n:
        k = n.split('::')[1].split('(')[0]
        acc[k][0] += 1; acc[k][1] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6
for k, (c, t) in sorted(acc.items(), key=lambda x: -x[1][1]):
    print(f"{k:28s} {c:5d} {t:9.3f} ms  avg {t / c * 1e3:9.1f} us")
PY
