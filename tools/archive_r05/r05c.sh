# r05c: the row kernel's dynamics balanced onto the longwave side (SML_DYN_BALANCE): sub-phase
# stamps, then same-box bench A/B (alternating), then the physics tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r05c
export SML_LIB_PST=abx/pst/speedy-ml-1_amd/lib/libspeedyml.so
for b in 1 0; do
  SML_DYN_BALANCE=$b SML_LIB=$SML_LIB_PST timeout -k 10 120 python -u tools/probe_pst.py > gpurun_out/r05c/pst_$b.txt 2>&1 || exit 1
  echo "balance=$b"; cat gpurun_out/r05c/pst_$b.txt | grep -v amdgpu.ids
done
B="bench.py --no-cpu-baseline --train-regions 0 --reservoir-steps 0 --speedy-steps 24 --steps 200 --warmup 10"
for rep in 1 2; do
  for b in 1 0; do
    SML_DYN_BALANCE=$b timeout -k 10 300 python -u $B > gpurun_out/r05c/ab_${b}_$rep.json 2> gpurun_out/r05c/ab_${b}_$rep.err || { tail gpurun_out/r05c/ab_${b}_$rep.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/r05c/ab_${b}_$rep.json').read().strip().splitlines()[-1]); s=d['speedy_step']; print('balance=$b rep $rep', d['value'], d['ms_per_step'], 'window', s['window_ms_graph_physics'], 'phys', s['roofline']['k_st_gridspec']['phases_us'])"
  done
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_physics_gpu.py tests/test_window_ref_gpu.py > gpurun_out/r05c/tests.log 2>&1; rc=$?; tail -2 gpurun_out/r05c/tests.log; exit $rc
