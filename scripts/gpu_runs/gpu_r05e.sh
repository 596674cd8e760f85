#!/bin/bash
# round 5 (e): GEMM tile / split-K sweep of the diffusion-phase (2,048-row) and projection shapes
set -o pipefail
mkdir -p gpurun_out
S="train_h,train_out,dh (NN),dW2,dW1,proj_v,dout+=G"
for nb in 0 1 2 3; do
  echo "=== GMR_GEMM_X6_NB128=$nb" >> gpurun_out/r05e_gemm.txt
  GMR_GEMM_X6_NB128=$nb timeout -k 10 200 python -u scripts/gemm_bench.py --only "$S" --mfma 6 --tiles 0,128 --splits 0,1,2,3,4 --reps 10 >> gpurun_out/r05e_gemm.txt 2>&1 || exit $?
done
echo "=== other tiles, x6 and fp32" >> gpurun_out/r05e_gemm.txt
timeout -k 10 300 python -u scripts/gemm_bench.py --only "$S" --mfma 6,32 --tiles 64,256128,128256,256 --splits 0,1,2,4 --reps 10 >> gpurun_out/r05e_gemm.txt 2>&1
