#!/bin/bash
# round 6 (q): tile sweep of the split-bf16 kernel (two accumulator sets) on the DiffMM x6 shapes, to re-tune the
# automatic plan after the 128^2 three-blocks-per-CU tile became opt-in
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u scripts/gemm_bench.py --tiles 0,128,256128,128256,256 --mfma 6 --reps 10 \
  --only psample,train_h,train_out,dh,dW2,dW1 2>&1 | grep -v amdgpu.ids > gpurun_out/r06q_x6_tiles.txt || exit 1
GMR_GEMM_X6_NB128=3 timeout -k 10 300 python -u scripts/gemm_bench.py --tiles 128 --mfma 6 --reps 10 \
  --only psample,train_h,train_out,dh,dW2,dW1 2>&1 | grep -v amdgpu.ids >> gpurun_out/r06q_x6_tiles.txt || exit 1
cat gpurun_out/r06q_x6_tiles.txt
echo all-done
