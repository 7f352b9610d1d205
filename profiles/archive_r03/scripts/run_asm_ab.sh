# r03d: the one-rank finish that also assembles the grids (sml_res_step_finish_assemble
# inside sml_hybrid_step) -- bitwise tests, then the headline A/B (SML_HYBRID_ASM=0:
# the separate assembly)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_reservoir_gpu.py tests/test_hybrid_gpu.py tests/test_fortran_hybrid_gpu.py > gpurun_out/asm_tests.log 2>&1
rc=$?; grep -E "passed|failed|Error" gpurun_out/asm_tests.log | tail -3; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for a in 0 1; do
    SML_HYBRID_ASM=$a timeout -k 10 200 python -u bench.py --no-cpu-baseline --train-regions 0 --speedy-steps 0 --reservoir-steps 0 > gpurun_out/asm_$a$i.json 2> gpurun_out/asm_$a$i.err || { tail -5 gpurun_out/asm_$a$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/asm_$a$i.json').read().strip().splitlines()[-1]); print('SML_HYBRID_ASM=$a rep $i', d['value'], d['ms_per_step'])"
  done
done
