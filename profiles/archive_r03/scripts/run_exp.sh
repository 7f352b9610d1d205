# r03: physics / window tests, phase-contention probes of A ($SML_LIB_A) and the
# tree's build, partner-memory probes, then the same-box headline A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_physics_gpu.py tests/test_window_ref_gpu.py -x -q --timeout 240 --timeout-method thread > gpurun_out/exp_tests.log 2>&1
rc=$?; tail -2 gpurun_out/exp_tests.log; [ $rc -eq 0 ] || exit $rc
SML_LIB=$SML_LIB_A timeout -k 10 200 python -u tools/probe_phase_contention.py > gpurun_out/exp_pc_A.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/probe_phase_contention.py > gpurun_out/exp_pc_B.log 2>&1 || exit 1
for m in uncached finegrained; do PARTNER_MEM=$m timeout -k 10 200 python -u tools/probe_phase_contention.py > gpurun_out/exp_pc_$m.log 2>&1 || exit 1; done
N=${N:-3} bash profiles/run_ab.sh
