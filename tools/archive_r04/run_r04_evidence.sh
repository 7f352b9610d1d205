# round 4 evidence at HEAD: the full -m gpu suite, smoke(), the default bench line,
# the driver's command, and the rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE passes
set -o pipefail
R=${1:-r04a}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/${R}_gpu_tests.log 2>&1
rc=$?
echo "pytest rc $rc" >> gpurun_out/${R}_gpu_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${R}_smoke.log 2>&1 || exit 3
timeout -k 10 400 python bench.py > gpurun_out/${R}_bench.json 2> gpurun_out/${R}_bench.err || exit 4
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${R}_bench_driver.json 2> gpurun_out/${R}_bench_driver.err || exit 5
timeout -k 10 1000 bash profiles/collect.sh $R > gpurun_out/collect_$R.log 2>&1 || exit 6
