#!/bin/bash
# round 5 (ze): DiffMM diffusion phase with independent denoiser chains (GMR_INDEP_DENOISERS): tests, A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_phases_gpu.py \
  tests/test_diffmm_gpu.py tests/test_resume_gpu.py tests/test_dist_gpu.py > gpurun_out/r05ze_tests.log 2>&1 || exit $?
for cfg in "GMR_INDEP_DENOISERS=0" "GMR_INDEP_DENOISERS=1" "GMR_INDEP_DENOISERS=0" "GMR_INDEP_DENOISERS=1" "GMR_INDEP_DENOISERS=0" "GMR_INDEP_DENOISERS=1"; do
  echo "=== $cfg" >> gpurun_out/r05ze_ab.txt
  env $cfg GMR_PHASE_TIMES=1 timeout -k 10 200 python -u bench.py --model diffmm --no-legs --no-cpu-baseline --no-probe --steps 5 --warmup 1 2>gpurun_out/r05ze_err.txt | cut -c1-200 >> gpurun_out/r05ze_ab.txt || exit $?
  grep phases gpurun_out/r05ze_err.txt | tail -2 >> gpurun_out/r05ze_ab.txt
done
