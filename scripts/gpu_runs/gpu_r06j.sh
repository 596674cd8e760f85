#!/bin/bash
# round 6 (j): split accumulators in the split-bf16 GEMM (hi*hi apart from the five small products) and the
# InfoNCE Y products on three split terms.  ablibs/libgmr_head.so = HEAD's gemm_x6.hip, libgmr_two.so = split
# accumulators, libgmr_y3.so = split accumulators + Y3 (all three read the batch rows in place).  MFMA rounding
# micro, bias probe, gc rows vs fp64, kernel tests, per-shape GEMM time, epoch A/B.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 ./scripts/micro/mfma_round 20000 > gpurun_out/r06j_mfma_rounding.txt || exit $?
for v in two head; do
  export GMR_HIP_LIB=$PWD/ablibs/libgmr_$v.so
  echo "=== $v"
  timeout -k 10 120 python -u scripts/x6_bias_probe.py 2>&1 | grep -v amdgpu.ids || exit $?
  timeout -k 10 300 python -u -m pytest -q -s --timeout 200 --timeout-method thread tests/test_diffmm_train_gpu.py -m gpu \
    -k "diffusion_step" > gpurun_out/r06j_gc_$v.log 2>&1; rc=$?; [ $rc -ge 124 ] && exit $rc
  grep -E "^\[|passed|failed" gpurun_out/r06j_gc_$v.log
  timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "x6 or gemm or contrast" \
    > gpurun_out/r06j_x6_$v.log 2>&1; rc=$?; tail -1 gpurun_out/r06j_x6_$v.log; [ $rc -ge 124 ] && exit $rc
  timeout -k 10 200 python -u scripts/gemm_bench.py --tiles 0 --reps 20 2>&1 | grep -v amdgpu.ids > gpurun_out/r06j_gemm_$v.txt || exit $?
done
paste gpurun_out/r06j_gemm_two.txt gpurun_out/r06j_gemm_head.txt | cut -c1-160
export GMR_HIP_LIB=$PWD/ablibs/libgmr_y3.so
echo "=== y3"
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_diffmm_train_gpu.py \
  tests/test_diffmm_gpu.py tests/test_stream_order_gpu.py tests/test_genrec_gpu.py -m gpu -k "contrast or rec_step or train or infonce or stream or epochs" \
  > gpurun_out/r06j_y3_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r06j_y3_tests.log; [ $rc -ge 124 ] && exit $rc
timeout -k 10 120 python -u scripts/contrast_bench.py 2>&1 | grep -v amdgpu.ids
export GMR_HIP_LIB=$PWD/ablibs/libgmr_two.so
timeout -k 10 120 python -u scripts/contrast_bench.py 2>&1 | grep -v amdgpu.ids
for v in two head y3 two head y3; do
  export GMR_HIP_LIB=$PWD/ablibs/libgmr_$v.so
  echo "=== $v" >> gpurun_out/r06j_ab.txt
  GMR_PHASE_TIMES=1 timeout -k 10 200 python -u bench.py --model diffmm --no-legs --no-cpu-baseline --no-probe --steps 5 --warmup 1 2>gpurun_out/r06j_err.txt | cut -c1-200 >> gpurun_out/r06j_ab.txt || exit $?
  grep phases gpurun_out/r06j_err.txt | tail -3 >> gpurun_out/r06j_ab.txt
done
cat gpurun_out/r06j_ab.txt
echo all-done
