# rocprof evidence (trace + FETCH/WRITE passes) and a timeline of one hybrid step
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash profiles/collect.sh ${R:-r01l} || exit $?
f=$(ls gpurun_out/prof_${R:-r01l}/trace/*kernel_trace.csv | head -1)
python3 tools/trace_timeline.py "$f" k_res_readout 30 2 60 > gpurun_out/timeline_${R:-r01l}.txt
cat gpurun_out/timeline_${R:-r01l}.txt | head -70
