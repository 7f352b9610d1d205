# r05x: run_model's exit inside the window graph -- run_model / hybrid / sharded / slab tests, A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r05x
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_run_model_gpu.py tests/test_hybrid_gpu.py tests/test_sharded_gpu.py tests/test_slab_gpu.py tests/test_force_exchange_gpu.py tests/test_fortran_hybrid_gpu.py tests/test_window_ref_gpu.py > gpurun_out/r05x/tests.log 2>&1 || { tail -30 gpurun_out/r05x/tests.log; exit 1; }
tail -1 gpurun_out/r05x/tests.log
bash tools/gpu/ab_bench.sh r05x/ab "SML_HOP_DONE=1" "SML_HOP_DONE=0" "SML_HOP_FUSED=1" "SML_HOP_DONE=0 SML_EXIT_GRAPH=0"
o=$GRAFT_REPO_ROOT/gpurun_out/r05x; export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $o/prof -o run --output-format csv -- python3 -u $GRAFT_REPO_ROOT/bench.py --sim-ranks 8 --no-cpu-baseline --train-regions 0 --steps 12 --warmup 3) > $o/b.json 2> $o/b.err || { tail $o/b.err; exit 1; }
python3 tools/trace_timeline.py $o/prof/run_kernel_trace.csv k_io_entry 10 8 8 > $o/timeline.txt
cat $o/timeline.txt
