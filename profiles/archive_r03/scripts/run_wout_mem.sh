# r03: the readout's W_out memory type (SML_WOUT_MEM) vs SPEEDY's window beside it
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for m in default uncached coherent; do
  SML_WOUT_MEM=$m timeout -k 10 300 python -u tools/probe_contention.py > gpurun_out/contention_$m.log 2>&1 || { tail -5 gpurun_out/contention_$m.log; exit 1; }
  echo "== $m"; grep -E "window|alone" gpurun_out/contention_$m.log | head -4
done
