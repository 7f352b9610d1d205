#!/bin/bash
# r04e2: the chain-mode test against the committed build (hop kernels) and the tree's
set -o pipefail
mkdir -p gpurun_out/r04e2
T="timeout -k 10"
SML_LIB=$PWD/ablib/libspeedyml_0edeac5.so $T 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_hybrid_gpu.py -k chain_on_speedys > gpurun_out/r04e2/head.log 2>&1; echo "head rc=$?"; tail -3 gpurun_out/r04e2/head.log
$T 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_hybrid_gpu.py -k chain_on_speedys > gpurun_out/r04e2/tree.log 2>&1; echo "tree rc=$?"; tail -3 gpurun_out/r04e2/tree.log
