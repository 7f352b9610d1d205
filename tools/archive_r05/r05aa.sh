# r05aa: the tile GEMMs' epilogue reads batched per MFMA row -- bitwise vs HEAD's build, tests, same-box A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"; o=gpurun_out/r05aa; mkdir -p $o
OLD=$GRAFT_REPO_ROOT/abx/old/speedy-ml-1_amd/lib/libspeedyml.so
SML_LIB=$OLD timeout -k 10 120 python -u tools/train_dump.py $o/w_old.npy > $o/dump_old.log 2>&1 || { tail $o/dump_old.log; exit 1; }
timeout -k 10 120 python -u tools/train_dump.py $o/w_new.npy > $o/dump_new.log 2>&1 || { tail $o/dump_new.log; exit 1; }
python3 -c "import numpy as np; a=np.load('$o/w_old.npy'); b=np.load('$o/w_new.npy'); print('bitwise', np.array_equal(a,b), 'max diff', abs(a-b).max())"
bash tools/gpu/ab_train.sh r05aa/ab "SML_LIB=$OLD" "SML_X=1"
