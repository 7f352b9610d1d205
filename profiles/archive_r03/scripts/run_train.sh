# r03: training GPU tests + the training leg (default kernels)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_training_gpu.py -x -q --timeout 250 --timeout-method thread > gpurun_out/r03_train_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r03_train_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --reservoir-steps 0 --speedy-steps 0 --no-cpu-baseline > gpurun_out/r03_train.json 2> gpurun_out/r03_train.err || { tail -5 gpurun_out/r03_train.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r03_train.json').read().strip().splitlines()[-1])['training']; print('gram', d['gram_ms'], d['roofline']['achieved'], d['roofline']['frac'], 'solve', d['solve_ms'], d['solve_roofline']['achieved'], d['solve_roofline']['frac'], d['solve_info_ok'])"
