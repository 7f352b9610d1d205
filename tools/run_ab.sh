# A/B of two builds of libspeedyml.so (A: lib/, B: $SML_LIB_B) on the default short bench, alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/ab
timeout -k 10 300 python -u -m pytest tests/test_hybrid_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/test.log 2>&1 || { tail -30 gpurun_out/ab/test.log; exit 1; }
tail -1 gpurun_out/ab/test.log
B="bench.py --no-cpu-baseline --train-regions 0 --reservoir-steps 0 --speedy-steps 0 --steps 60"
for i in 1 2 3; do for v in A B; do
  if [ $v = B ]; then export SML_LIB=$GRAFT_REPO_ROOT/$SML_LIB_B; else unset SML_LIB; fi
  timeout -k 10 200 python -u $B > gpurun_out/ab/$v$i.json 2> gpurun_out/ab/$v$i.err || { tail gpurun_out/ab/$v$i.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ab/$v$i.json').read().strip().splitlines()[-1]); print('$v$i', d['value'], d['ms_per_step'], d['roofline']['achieved'], d['roofline']['readout_avg_ms'])"
done; done
