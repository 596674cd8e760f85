#!/bin/bash
# round 6 (o): vectorised arg-max rows (four columns per load) + SCALE_BIAS last p_sample step without the env
# switch: top-K / rebuild / p_sample tests, then the rebuild's kernel durations (one epoch, serial streams)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_kernels_gpu.py \
  tests/test_psample_fold_gpu.py tests/test_baby_gpu.py tests/test_diffmm_gpu.py tests/test_diffrec_baby_gpu.py -k "topk or argmax or psample or rebuild or baby or fold or scale_bias" \
  > gpurun_out/r06o_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r06o_tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/r06o_tests.log | head -20; exit 1; }
GMR_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06o_prof -o prof -- python3 bench.py --no-legs --no-cpu-baseline --no-probe --steps 1 --warmup 1 > gpurun_out/r06o_prof.log 2>&1 || exit 1
grep -E "argmax_rows|densify|gemm_x6_kernel<128" gpurun_out/r06o_prof/prof_kernel_stats.csv | cut -c1-160
echo all-done
