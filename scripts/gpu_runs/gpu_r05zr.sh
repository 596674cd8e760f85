#!/bin/bash
# round 5 (zr): split-bf16 TN / NN operands read in place (no x6_transpose copies): tests, then the
# denoiser / decoder gradient products with GMR_X6_INPLACE = 0 (copies) and 1 (in place)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "x6 or glds" -m gpu > gpurun_out/r05zr_tests.log 2>&1 || exit $?
for v in 0 1 0 1; do
  echo "=== GMR_X6_INPLACE=$v" >> gpurun_out/r05zr_bench.txt
  GMR_X6_INPLACE=$v timeout -k 10 200 python -u scripts/gemm_bench.py --only "dh (NN),dW2,dW1,tf_dg,tf_dWout,tf_dWin" \
    --tiles 0 --mfma 6 >> gpurun_out/r05zr_bench.txt 2>&1 || exit $?
done
