#!/bin/bash
# SpMM lane plans with non-temporal index loads / Y stores (GMR_SPMM_NT = 0..3).
set -o pipefail
TAG=${1:-r02i}
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
for NT in 0 1 2 3; do
GMR_SPMM_NT=$NT timeout -k 10 200 python scripts/spmm_bench.py --segs 65568,196640 --nbs 1,2,4 --graphs norm_adj,ui_top1 --reps 50 > gpurun_out/${TAG}_spmm_nt$NT.txt 2>&1; rc=$?
echo "== NT $NT"; grep -v amdgpu gpurun_out/${TAG}_spmm_nt$NT.txt | tail -14; fatal $rc spmm
done
echo all-done
