# round-2 GPU evidence: every GPU test, smoke(), the default bench line, rocprof trace
# usage (on the box): R=r02a bash profiles/run_r02.sh [tests|bench|prof ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
R=${R:-r02a}
for what in "$@"; do
  case $what in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${R}_gpu_tests.log 2>&1
      rc=$?; tail -3 gpurun_out/${R}_gpu_tests.log; [ $rc -eq 0 ] || exit $rc ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${R}_smoke.log 2>&1 || { tail -20 gpurun_out/${R}_smoke.log; exit 1; }
      tail -1 gpurun_out/${R}_smoke.log ;;
    bench)
      timeout -k 10 600 python -u bench.py > gpurun_out/${R}_bench.json 2> gpurun_out/${R}_bench.err || { tail -20 gpurun_out/${R}_bench.err; exit 1; }
      tail -1 gpurun_out/${R}_bench.json ;;
    quick)
      timeout -k 10 300 python -u bench.py --no-cpu-baseline --train-regions 0 --speedy-steps 8 --reservoir-steps 10 > gpurun_out/${R}_quick.json 2> gpurun_out/${R}_quick.err || { tail -20 gpurun_out/${R}_quick.err; exit 1; }
      tail -1 gpurun_out/${R}_quick.json ;;
    prof)
      bash profiles/collect.sh $R > gpurun_out/${R}_collect.log 2>&1 || { tail -20 gpurun_out/${R}_collect.log; exit 1; }
      echo collect ok ;;
  esac
done
