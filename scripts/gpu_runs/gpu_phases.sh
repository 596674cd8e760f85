#!/bin/bash
# Phase wall times of the DiffMM epoch, per-shape probe report, and p_sample GEMM shapes at 19k rows.
set -o pipefail
TAG=${1:-phases}
mkdir -p gpurun_out
export TMPDIR=/tmp
GMR_PHASE_TIMES=1 GMR_PROBE_REPORT=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-legs > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo bench failed; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
grep -E "phases|warmup" gpurun_out/${TAG}_bench.err | head -20
timeout -k 10 200 python scripts/gemm_bench.py --only "psample_h19k,psample_out19k" --tiles 128,256,256128 --splits 1,2 --reps 5 > gpurun_out/${TAG}_gemm.txt 2>&1; cat gpurun_out/${TAG}_gemm.txt | grep -v amdgpu
echo all-done
