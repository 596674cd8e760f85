#!/bin/bash
# split-bf16 GEMM timing under several environment settings (A/B): one gemm_bench pass per setting
# usage: scripts/gpu_x6_env.sh <tag> <shape filter> <tiles> "<ENV=a ENV2=b>" "<ENV=c>" ...
set -o pipefail
TAG=$1; ONLY=$2; TILES=$3; shift 3
mkdir -p gpurun_out
export TMPDIR=/tmp
for setting in "$@"; do
  echo "--- $setting"
  env $setting timeout -k 10 200 python scripts/gemm_bench.py --only "$ONLY" --tiles $TILES --mfma 6 --reps 10 > gpurun_out/${TAG}.txt 2>&1 || { tail -5 gpurun_out/${TAG}.txt; exit 1; }
  grep " m6 " gpurun_out/${TAG}.txt
done
