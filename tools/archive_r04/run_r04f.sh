# round 4: the training GEMMs on v_mfma_f64_4x4x4_f64
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_training_gpu.py > gpurun_out/t6.log 2>&1
echo "pytest rc $?" >> gpurun_out/t6.log
timeout -k 10 300 python bench.py --no-cpu-baseline --reservoir-steps 0 --speedy-steps 0 --steps 50 > gpurun_out/g_train.json 2> gpurun_out/g_train.err || exit 3
