# r05z: vdifsc on the longwave side on longwave-only steps -- physics / window tests, A/B, sub-phase stamps
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r05z
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_physics_gpu.py tests/test_window_ref_gpu.py tests/test_dynamics_gpu.py > gpurun_out/r05z/tests.log 2>&1 || { tail -30 gpurun_out/r05z/tests.log; exit 1; }
tail -1 gpurun_out/r05z/tests.log
bash tools/gpu/ab_bench.sh r05z/ab "SML_VDIF_LW=1" "SML_VDIF_LW=0" || exit 1
for v in 1 0; do SML_VDIF_LW=$v SML_LIB=$GRAFT_REPO_ROOT/abx/pst/speedy-ml-1_amd/lib/libspeedyml.so timeout -k 10 120 python -u tools/probe_pst.py > gpurun_out/r05z/pst_$v.txt 2>&1 || { tail gpurun_out/r05z/pst_$v.txt; exit 1; }; echo "== SML_VDIF_LW=$v"; grep -E "done at|side" gpurun_out/r05z/pst_$v.txt; done
