#!/bin/bash
# round 6 (n): the last p_sample step as GMR_EPI_SCALE_BIAS (no aux read, no densified histories in the folded
# rebuild / DiffRec eval): the GEMM / p_sample / rebuild / DiffRec tests, then the epoch A/B
# (GMR_PSAMPLE_SCALE_BIAS=1 vs 0) for DiffMM and the DiffRec leg
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_kernels_gpu.py \
  tests/test_psample_fold_gpu.py tests/test_baby_gpu.py tests/test_diffrec_gpu.py tests/test_diffrec_baby_gpu.py \
  tests/test_diffmm_gpu.py tests/test_phases_gpu.py tests/test_sports_gpu.py > gpurun_out/r06n_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r06n_tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/r06n_tests.log | head -20; exit 1; }
for v in 1 0 1 0; do
  echo "=== GMR_PSAMPLE_SCALE_BIAS=$v" >> gpurun_out/r06n_ab.txt
  GMR_PSAMPLE_SCALE_BIAS=$v GMR_PHASE_TIMES=1 timeout -k 10 200 python -u bench.py --model diffmm --no-legs --no-cpu-baseline --no-probe --steps 5 --warmup 1 2>gpurun_out/r06n_err.txt | cut -c1-200 >> gpurun_out/r06n_ab.txt || exit $?
  grep phases gpurun_out/r06n_err.txt | tail -3 >> gpurun_out/r06n_ab.txt
done
cat gpurun_out/r06n_ab.txt
echo all-done
