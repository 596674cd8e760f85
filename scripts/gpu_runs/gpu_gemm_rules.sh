#!/bin/bash
# GEMM tile/split rules: the rebuild/diffusion shapes per tile (auto split) and the DiffMM bench with
# the per-shape serial GEMM table.
set -o pipefail
TAG=${1:-r02f}
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
timeout -k 10 400 python scripts/gemm_bench.py --only "psample_post,psample_out (,train_out,dW,dh,proj_,train_Z" --tiles 0,64,128,256,256128 --reps 10 > gpurun_out/${TAG}_gemm.txt 2>&1; rc=$?
grep -v amdgpu gpurun_out/${TAG}_gemm.txt; fatal $rc gemm
GMR_PHASE_TIMES=1 GMR_PROBE_REPORT=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-legs > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err; rc=$?
head -c 400 gpurun_out/${TAG}_bench.json; echo; grep -B2 -A24 "gemm:" gpurun_out/${TAG}_bench.err; grep phase gpurun_out/${TAG}_bench.err; fatal $rc bench
echo all-done
