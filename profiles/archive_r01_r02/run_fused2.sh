# dynamics GPU tests, phase probe, then bench with the fused and the unfused step
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_physics_gpu.py tests/test_dynamics_gpu.py -m gpu -v -x --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log; tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/probe_phases.py 1 2>&1 | grep -v amdgpu.ids | tail -2 || exit $?
timeout -k 10 120 python -u tools/probe_phases.py 0 2>&1 | grep -v amdgpu.ids | tail -2 || exit $?
for fz in 1 0; do
SML_DYN_FUSED=$fz timeout -k 10 400 python -u bench.py --no-cpu-baseline --train-regions 0 > gpurun_out/bench_f$fz.json 2> gpurun_out/bench_f$fz.err || exit $?
python3 -c "
import json; d=json.loads(open('gpurun_out/bench_f$fz.json').read().strip().splitlines()[-1])
print('fused=$fz value', d['value'], 'ms', d['ms_per_step'], 'window', d['speedy_step']['window_ms_graph_physics'], d['speedy_step'])"
done
