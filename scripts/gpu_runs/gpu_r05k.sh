#!/bin/bash
# round 5 (k): multi-job side-split SpMM launches - bit-exactness tests, epoch A/B (side jobs off / on / + BWD3 fusion)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py::test_spmm_side_jobs_one_launch_bit_exact \
  tests/test_kernels_gpu.py::test_spmm_side_multi_outputs_and_jobs tests/test_diffmm_gpu.py tests/test_diffmm_baby_train_gpu.py \
  tests/test_sports_gpu.py > gpurun_out/r05k_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/r05k_tests.log
[ $rc -ne 0 ] && exit $rc
for cfg in "GMR_SPMM_SIDE_JOBS=0" "GMR_SPMM_SIDE_JOBS=1" "GMR_SPMM_FUSE=5" "GMR_SPMM_SIDE_JOBS=0" "GMR_SPMM_SIDE_JOBS=1" "GMR_SPMM_FUSE=5"; do
  echo "=== $cfg" >> gpurun_out/r05k_ab.txt
  env $cfg timeout -k 10 200 python -u bench.py --model diffmm --no-legs --no-cpu-baseline --no-probe --steps 5 --warmup 1 2>/dev/null | cut -c1-200 >> gpurun_out/r05k_ab.txt || exit $?
done
