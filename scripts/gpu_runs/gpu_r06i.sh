#!/bin/bash
# round 6 (i): two-level accumulation in the split-bf16 GEMM (per-k-tile partial sums, RNE fold): bias probe,
# gc rows vs fp64, x6 accuracy tests, per-shape GEMM time and epoch time, against the previous kernel
# (ablibs/libgmr_head.so = HEAD's gemm_x6.hip, ablibs/libgmr_two.so = the working tree's)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in two head; do
  export GMR_HIP_LIB=$PWD/ablibs/libgmr_$v.so
  echo "=== $v"
  timeout -k 10 120 python -u scripts/x6_bias_probe.py 2>&1 | grep -v amdgpu.ids || exit $?
  timeout -k 10 300 python -u -m pytest -q -s --timeout 200 --timeout-method thread tests/test_diffmm_train_gpu.py -m gpu \
    -k "diffusion_step" > gpurun_out/r06i_gc_$v.log 2>&1
  grep -E "^\[|passed|failed" gpurun_out/r06i_gc_$v.log
  timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "x6 or gemm" \
    > gpurun_out/r06i_x6_$v.log 2>&1; tail -1 gpurun_out/r06i_x6_$v.log
  timeout -k 10 200 python -u scripts/gemm_bench.py --tiles 0 --reps 20 2>&1 | grep -v amdgpu.ids > gpurun_out/r06i_gemm_$v.txt || exit $?
done
paste gpurun_out/r06i_gemm_two.txt gpurun_out/r06i_gemm_head.txt | cut -c1-160
for v in two head two head; do
  export GMR_HIP_LIB=$PWD/ablibs/libgmr_$v.so
  echo "=== $v" >> gpurun_out/r06i_ab.txt
  GMR_PHASE_TIMES=1 timeout -k 10 200 python -u bench.py --model diffmm --no-legs --no-cpu-baseline --no-probe --steps 5 --warmup 1 2>gpurun_out/r06i_err.txt | cut -c1-200 >> gpurun_out/r06i_ab.txt || exit $?
  grep phases gpurun_out/r06i_err.txt | tail -3 >> gpurun_out/r06i_ab.txt
done
cat gpurun_out/r06i_ab.txt
echo all-done
