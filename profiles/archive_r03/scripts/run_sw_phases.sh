# r03d: the window's last-step phases when that step is a shortwave step (NLEAP=22)
# and when it is not (NLEAP=24), alone and beside torch.sum
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for n in 24 22; do
  NLEAP=$n timeout -k 10 200 python -u tools/probe_phase_contention.py > gpurun_out/sw_$n.log 2>&1 || { tail -5 gpurun_out/sw_$n.log; exit 1; }
  echo "== NLEAP=$n"; grep -vE "amdgpu.ids" gpurun_out/sw_$n.log
done
