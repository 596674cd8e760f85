#!/bin/bash
# round 6 (g): rounding bias of the split-bf16 vs fp32-MFMA GEMM on the denoiser output-layer product
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/x6_bias_probe.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r06g_bias.txt
