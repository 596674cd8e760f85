#!/bin/bash
# Baby-shape parity tests + GEMM MFMA-shape sweep (32x32x2 vs 16x16x4) + full GPU test suite.
set -o pipefail
TAG=${1:-r02b}
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
timeout -k 10 300 python scripts/gemm_bench.py --only "train_h,dh (NN),train_out,dW2,psample_h (NT),psample_out (NT)" --tiles 64,128,256,256128 --mfma 32,16 --splits 1,2,4,8 --reps 10 > gpurun_out/${TAG}_gemm.txt 2>&1; rc=$?; fatal $rc gemm
tail -3 gpurun_out/${TAG}_gemm.txt
timeout -k 10 600 python -u -m pytest tests -v -m gpu -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
tail -3 gpurun_out/${TAG}_tests.log; grep -E "FAILED|ERROR" gpurun_out/${TAG}_tests.log | head; fatal $rc tests
echo all-done
