# r03d: specy's vfm loads first (SML_SPEC_VFM_FIRST, ab/vf1) vs the same source
# without (ab/vf0) and HEAD (tree): window tests on vf1, phase probe, headline A/B;
# then the step timeline of HEAD
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TESTED="vf1" VARIANTS="tree vf0 vf1" REPS=2 bash profiles/r03d/run_window_variants.sh || exit $?
timeout -k 10 200 python -u tools/probe_step_timeline.py > gpurun_out/r03d_timeline.log 2>&1 || { tail -5 gpurun_out/r03d_timeline.log; exit 1; }
grep -v amdgpu gpurun_out/r03d_timeline.log
