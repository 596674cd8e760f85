#!/bin/bash
# glds GEMM staging: parity tests, per-shape timing with and without it, and the DiffMM bench A/B.
set -o pipefail
TAG=${1:-r02k}
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread -k "gemm" > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_tests.log; grep -E "FAILED|ERROR" gpurun_out/${TAG}_tests.log | head -20; fatal $rc tests
for G in ${GLDS_SET:-1 0}; do
GMR_GEMM_GLDS=$G timeout -k 10 300 python scripts/gemm_bench.py --only "square8192,psample,train_,dh,dW,proj_v" --tiles 0,128,256,256128 --reps 10 > gpurun_out/${TAG}_gemm_g$G.txt 2>&1; rc=$?
echo "== GLDS $G"; grep -v amdgpu gpurun_out/${TAG}_gemm_g$G.txt; fatal $rc gemm
done
for G in ${GLDS_SET:-1 0}; do
GMR_GEMM_GLDS=$G GMR_PHASE_TIMES=1 GMR_PROBE_REPORT=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-legs > gpurun_out/${TAG}_bench_g$G.json 2> gpurun_out/${TAG}_bench_g$G.err; rc=$?
echo "== bench GLDS $G"; head -c 300 gpurun_out/${TAG}_bench_g$G.json; echo; grep -A12 "gemm:" gpurun_out/${TAG}_bench_g$G.err; grep phases gpurun_out/${TAG}_bench_g$G.err | tail -1; fatal $rc bench
done
echo all-done
