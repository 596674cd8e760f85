#!/bin/bash
# round 3: split-bf16 GEMM split-K / pipeline sweep on the rebuild and diffusion shapes
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/gemm_bench.py --tiles 0 --mfma 6 --splits 0,1,2,3,4 --only "psample_h19k,psample_out19k,train_h,train_out,dh,dW" > gpurun_out/r03s_split.txt 2>&1 || exit $?
GMR_GEMM_X6_PIPE=1 timeout -k 10 300 python -u scripts/gemm_bench.py --tiles 0,256128 --mfma 6 --only "psample_h19k,psample_out19k,train_h,train_out" > gpurun_out/r03s_pipe.txt 2>&1
