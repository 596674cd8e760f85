#!/bin/bash
# split-bf16 GEMM (GMR_GEMM_X6) vs the fp32-MFMA kernel on the NT denoiser shapes: time and error vs fp64
# usage: scripts/gpu_x6.sh <tag> [shape filter] [tiles] [extra env assignments for the x6 pass]
set -o pipefail
TAG=${1:-r02x6}
ONLY=${2:-"square8192,psample_h19k,psample_out19k,psample_post (,train_h,train_out"}
TILES=${3:-0,128,256128,128256}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python scripts/gemm_bench.py --only "$ONLY" --tiles $TILES --mfma 32,6 --reps 10 --acc > gpurun_out/${TAG}_gemm.txt 2>&1; rc=$?
grep -v amdgpu gpurun_out/${TAG}_gemm.txt; [ $rc -eq 0 ] || exit $rc
exit 0
