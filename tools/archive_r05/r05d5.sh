# r05d5: 16-column sub-blocks in k_chol_diag_b (default) vs 32 (abx/sub32) vs k_chol_diag; stamps
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu/ab_train.sh r05d5 "SML_CHOL_DIAG=1" "SML_CHOL_DIAG=2" "SML_LIB=abx/sub32/speedy-ml-1_amd/lib/libspeedyml.so" || exit 1
SML_LIB=abx/dst/speedy-ml-1_amd/lib/libspeedyml.so timeout -k 10 200 python -u tools/probe_diag.py 10 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r05d5/stamps16.txt
