# r05a: the per-window forcing (sml_dyn_fordate), late hops, and the tests around them
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r05a
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 500 $T tests/test_fordate_gpu.py "tests/test_slab_gpu.py::test_slab_loop_date_forcing" \
    "tests/test_hybrid_gpu.py::test_a_hop_that_times_out_fails_the_step" \
    tests/test_physics_gpu.py tests/test_run_model_gpu.py tests/test_window_ref_gpu.py \
    "tests/test_fortran_hybrid_gpu.py::test_fortran_hybrid_driver_with_slab_matches_hybrid_loop" \
    "tests/test_reservoir_gpu.py::test_balanced_update_is_bitwise_the_per_region_update" \
    "tests/test_reservoir_gpu.py::test_ell_layouts_are_bitwise_the_csr_update" \
    > gpurun_out/r05a/test.log 2>&1
rc=$?
grep -E "PASS|FAIL|ERROR|fordate vs|slab loop|Error|assert" gpurun_out/r05a/test.log | tail -60
tail -3 gpurun_out/r05a/test.log
exit $rc
