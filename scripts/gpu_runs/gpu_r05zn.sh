#!/bin/bash
# round 5 (zn): projection GEMM shapes: tiles x MFMA shapes x split-K (the BPR step's critical-path products)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/gemm_bench.py --only proj_v --tiles 64,128 --mfma 32,16 --splits 0,4,8,16,32 --reps 30 > gpurun_out/r05zn_gemm.txt 2>&1 || exit $?
