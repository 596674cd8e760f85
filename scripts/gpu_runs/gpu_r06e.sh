#!/bin/bash
# round 6 (e): gc-row error diagnostics (denoiser output vs fp64, Z product vs exact), then the GPU suite after
# pruning the graph executor and the fused decoder
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q -s --timeout 200 --timeout-method thread tests/test_diffmm_train_gpu.py -m gpu \
  -k "diffusion_step_vs" > gpurun_out/r06e_gc.log 2>&1
grep -E "^\[|passed|failed" gpurun_out/r06e_gc.log
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu -k "not diffusion_step" \
  > gpurun_out/r06e_tests.log 2>&1 || { tail -60 gpurun_out/r06e_tests.log; exit 1; }
tail -2 gpurun_out/r06e_tests.log
echo done
