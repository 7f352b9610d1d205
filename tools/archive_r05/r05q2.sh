set -o pipefail
cd "$GRAFT_REPO_ROOT"; o=gpurun_out/r05q; mkdir -p $o
SML_LIB=abx/pst/speedy-ml-1_amd/lib/libspeedyml.so timeout -k 10 200 python -u tools/probe_pstq.py 2>&1 | tee $o/pstq.txt
