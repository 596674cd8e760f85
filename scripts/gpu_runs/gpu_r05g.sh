#!/bin/bash
# round 5 (g): pre-split InfoNCE staging - bit-exactness, fp64 accuracy, microbenchmark both ways; rec-step tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k contrast \
  tests/test_diffmm_gpu.py tests/test_diffmm_baby_train_gpu.py tests/test_genrec_gpu.py > gpurun_out/r05g_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/r05g_tests.log
[ $rc -ge 124 ] && exit $rc
for ps in 0 1; do
  echo "=== GMR_CL_PRESPLIT=$ps" >> gpurun_out/r05g_cl.txt
  GMR_CL_PRESPLIT=$ps timeout -k 10 120 python -u scripts/contrast_bench.py >> gpurun_out/r05g_cl.txt 2>&1 || exit $?
done
