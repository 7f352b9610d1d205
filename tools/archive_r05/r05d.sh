# r05d: rocprofv3 evidence of the default bench (kernel trace + FETCH / WRITE passes), and the
# FETCH_SIZE calibration probe at the update kernel's access widths (own passes)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r05d
export TMPDIR=/tmp
P=$GRAFT_REPO_ROOT/tools/probe_fetch_width
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r05d/probe_fetch -o probe --output-format csv -- $P) > gpurun_out/r05d/probe_fetch.log 2>&1 || { tail gpurun_out/r05d/probe_fetch.log; exit 1; }
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r05d/probe_write -o probe --output-format csv -- $P) > gpurun_out/r05d/probe_write.log 2>&1 || { tail gpurun_out/r05d/probe_write.log; exit 1; }
tail -1 gpurun_out/r05d/probe_fetch.log
bash profiles/collect.sh r05d
