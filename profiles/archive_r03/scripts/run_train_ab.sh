# r03: training kernels: GPU tests, then the training leg with k_train_gram2 (default) and k_train_gram (A/B)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_training_gpu.py -x -q --timeout 250 --timeout-method thread > gpurun_out/r03_train_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r03_train_tests.log; [ $rc -eq 0 ] || exit $rc
for v in 2 1; do
  SML_GRAM_V=$v timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --reservoir-steps 0 --speedy-steps 0 --no-cpu-baseline > gpurun_out/r03_train_v$v.json 2> gpurun_out/r03_train_v$v.err || { tail -5 gpurun_out/r03_train_v$v.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r03_train_v$v.json').read().strip().splitlines()[-1])['training']; print('gram v$v', d['gram_ms'], d['roofline']['achieved'], d['roofline']['frac_of_nominal_peak'], 'solve', d['solve_ms'], d['solve_roofline']['achieved'], d['solve_roofline']['frac_of_nominal_peak'], d['solve_info_ok'])"
done
