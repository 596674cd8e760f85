#!/bin/bash
# round 5 (zt): split-bf16 TN / NN operands read in place by single-float row loads (GMR_X6_INPLACE = 2, default),
# B only (1), copies (0): tests, the gradient products per mode, then epoch A/B 0 vs 2
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 170 --timeout-method thread tests/test_kernels_gpu.py \
  -k "x6 or glds" -m gpu > gpurun_out/r05zt_tests.log 2>&1 || exit $?
for v in 0 1 2; do
  echo "=== GMR_X6_INPLACE=$v" >> gpurun_out/r05zt_bench.txt
  GMR_X6_INPLACE=$v timeout -k 10 200 python -u scripts/gemm_bench.py --only "dh (NN),dW2,dW1,tf_dg,tf_dWout,tf_dWin" \
    --tiles 0 --mfma 6 2>&1 | grep -v amdgpu.ids >> gpurun_out/r05zt_bench.txt || exit $?
done
for v in 0 2 0 2; do
  echo "=== GMR_X6_INPLACE=$v" >> gpurun_out/r05zt_ab.txt
  GMR_X6_INPLACE=$v GMR_PHASE_TIMES=1 timeout -k 10 200 python -u bench.py --model diffmm --no-legs --no-cpu-baseline --no-probe --steps 5 --warmup 1 2>gpurun_out/r05zt_err.txt | cut -c1-200 >> gpurun_out/r05zt_ab.txt || exit $?
  grep phases gpurun_out/r05zt_err.txt | tail -2 >> gpurun_out/r05zt_ab.txt
done
