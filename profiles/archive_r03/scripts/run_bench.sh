# r03: the default bench line (args pass through), stdout JSON to gpurun_out/$OUT.json
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
OUT=${OUT:-r03_bench}
timeout -k 10 ${T:-900} python -u bench.py "$@" > gpurun_out/$OUT.json 2> gpurun_out/$OUT.err
rc=$?; tail -3 gpurun_out/$OUT.err; exit $rc
