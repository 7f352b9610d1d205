# r03d: which phases of the window grow beside a partner stream of each kind:
# torch.sum (plain loads), an nt-load read, a plain-load read (tools/libstream_partner.so)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for k in sum nt plain; do
  PARTNER_KIND=$k timeout -k 10 200 python -u tools/probe_phase_contention.py > gpurun_out/pk_$k.log 2>&1 || { tail -5 gpurun_out/pk_$k.log; exit 1; }
  echo "== $k"; grep -vE "amdgpu.ids" gpurun_out/pk_$k.log
done
