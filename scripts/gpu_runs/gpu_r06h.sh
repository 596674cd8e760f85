#!/bin/bash
# round 6 (h): gc-row error by GEMM path: default, hidden layer on fp32 MFMA, every product on fp32 MFMA
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for env in "GMR_X=0" "GMR_HIDDEN_F32=1" "GMR_GEMM_X6=0"; do
  echo "=== $env"
  env $env timeout -k 10 300 python -u -m pytest -q -s --timeout 200 --timeout-method thread tests/test_diffmm_train_gpu.py -m gpu \
    -k "diffusion_step_vs and baby" > gpurun_out/r06h_gc.log 2>&1
  grep -E "^\[|passed|failed" gpurun_out/r06h_gc.log
done
