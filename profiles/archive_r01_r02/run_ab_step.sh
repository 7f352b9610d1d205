# step-kernel parity tests, then a same-box A/B of the headline bench against the
# library in ab/$REV (tools/ab_build.sh REV), N alternations
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_physics_gpu.py tests/test_window_ref_gpu.py tests/test_dynamics_gpu.py tests/test_run_model_gpu.py tests/test_spectral_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab_tests.log 2>&1; rc=$?; tail -3 gpurun_out/ab_tests.log; [ $rc -eq 0 ] || exit $rc
SML_LIB_A=$PWD/ab/${REV:-HEAD}/speedy-ml-1_amd/lib/libspeedyml.so N=${N:-3} bash profiles/run_ab.sh || exit 1
for f in gpurun_out/ab_A1.json gpurun_out/ab_B1.json; do python3 -c "
import json; d=json.load(open('$f')); r=d['speedy_step']['roofline']; print('$f', r['k_st_gridspec']['phases_us'], r['k_st_spec']['span_us'], r['k_st_spec']['phases_us'])"; done
