#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python scripts/gemm_bench.py --only "proj_,train_Z,dout+=" --tiles 64,128 --splits 1,2,4,8,16,32,64 --reps 20 > gpurun_out/skinny_gemm.txt 2>&1; grep -v amdgpu gpurun_out/skinny_gemm.txt
