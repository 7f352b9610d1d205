# rocprof trace + FETCH/WRITE passes of the default bench, a timeline of one
# steady-state hybrid step, and the in-kernel phase stamps of the fused SPEEDY step
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
R=${R:-r02d}
bash profiles/collect.sh $R > gpurun_out/${R}_collect.log 2>&1 || { tail -20 gpurun_out/${R}_collect.log; exit 1; }
f=$(ls gpurun_out/prof_$R/trace/*kernel_trace.csv | head -1)
python3 tools/trace_timeline.py "$f" k_res_finish_grid 15 3 90 > gpurun_out/${R}_timeline.txt
head -100 gpurun_out/${R}_timeline.txt
timeout -k 10 300 python3 tools/probe_phases.py 1 > gpurun_out/${R}_phases.txt 2>&1 || { tail -20 gpurun_out/${R}_phases.txt; exit 1; }
cat gpurun_out/${R}_phases.txt
