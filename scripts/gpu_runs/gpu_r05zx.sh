#!/bin/bash
# round 5 (zx): gmr_zero as a 16-byte-store kernel vs hipMemsetAsync (GMR_ZERO_MEMSET=1): DiffMM tests, epoch A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_diffmm_gpu.py \
  tests/test_diffmm_baby_train_gpu.py tests/test_host_cpu.py -m gpu > gpurun_out/r05zx_tests.log 2>&1 || exit $?
for v in 1 0 1 0 1 0; do
  echo "=== GMR_ZERO_MEMSET=$v" >> gpurun_out/r05zx_ab.txt
  GMR_ZERO_MEMSET=$v GMR_PHASE_TIMES=1 timeout -k 10 200 python -u bench.py --model diffmm --no-legs --no-cpu-baseline --no-probe --steps 5 --warmup 1 2>gpurun_out/r05zx_err.txt | cut -c1-200 >> gpurun_out/r05zx_ab.txt || exit $?
  grep phases gpurun_out/r05zx_err.txt | tail -2 >> gpurun_out/r05zx_ab.txt
done
