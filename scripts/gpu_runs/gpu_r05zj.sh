#!/bin/bash
# round 5 (zj): modality projections as NT split-bf16 products (GMR_PROJ_X6 = 1 both / 2 image only): tests, A/B
set -o pipefail
mkdir -p gpurun_out
GMR_PROJ_X6=1 timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_diffmm_gpu.py \
  tests/test_diffmm_baby_train_gpu.py tests/test_phases_gpu.py > gpurun_out/r05zj_tests.log 2>&1 || exit $?
for cfg in "GMR_PROJ_X6=0" "GMR_PROJ_X6=1" "GMR_PROJ_X6=2" "GMR_PROJ_X6=0" "GMR_PROJ_X6=1" "GMR_PROJ_X6=2"; do
  echo "=== $cfg" >> gpurun_out/r05zj_ab.txt
  env $cfg GMR_PHASE_TIMES=1 timeout -k 10 200 python -u bench.py --model diffmm --no-legs --no-cpu-baseline --no-probe --steps 5 --warmup 1 2>gpurun_out/r05zj_err.txt | cut -c1-200 >> gpurun_out/r05zj_ab.txt || exit $?
  grep phases gpurun_out/r05zj_err.txt | tail -2 >> gpurun_out/r05zj_ab.txt
done
