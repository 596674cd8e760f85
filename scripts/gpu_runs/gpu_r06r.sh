#!/bin/bash
# round 6 (r): split-bf16 plans on 256 x 128 where they took 128^2 (the >= 768-tile rule and the large TN / NN
# gradients): GEMM / denoiser / training tests, per-shape times, and the epoch A/B against the previous library
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_kernels_gpu.py \
  tests/test_diffmm_train_gpu.py tests/test_psample_fold_gpu.py tests/test_baby_gpu.py tests/test_phases_gpu.py \
  tests/test_diffrec_baby_gpu.py -k "gemm or x6 or diffusion or train or psample or fold or baby or phase" > gpurun_out/r06r_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r06r_tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/r06r_tests.log | head -20; exit 1; }
for v in tile prev tile prev; do
  echo "=== $v" >> gpurun_out/r06r_ab.txt
  GMR_HIP_LIB=$PWD/ablibs/libgmr_$v.so GMR_PHASE_TIMES=1 timeout -k 10 200 python -u bench.py --model diffmm --no-legs --no-cpu-baseline --no-probe --steps 5 --warmup 1 2>gpurun_out/r06r_err.txt | cut -c1-200 >> gpurun_out/r06r_ab.txt || exit $?
  grep phases gpurun_out/r06r_err.txt | tail -3 >> gpurun_out/r06r_ab.txt
done
cat gpurun_out/r06r_ab.txt
echo all-done
