#!/bin/bash
# round 5 (zh): the two InfoNCE terms on one side stream (GMR_CL_ONE_STREAM): tests, A/B
set -o pipefail
mkdir -p gpurun_out
GMR_CL_ONE_STREAM=1 timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_diffmm_gpu.py \
  tests/test_graph_capture_gpu.py tests/test_diffmm_baby_train_gpu.py > gpurun_out/r05zh_tests.log 2>&1 || exit $?
for cfg in "GMR_CL_ONE_STREAM=0" "GMR_CL_ONE_STREAM=1" "GMR_CL_ONE_STREAM=0" "GMR_CL_ONE_STREAM=1" "GMR_CL_ONE_STREAM=0" "GMR_CL_ONE_STREAM=1"; do
  echo "=== $cfg" >> gpurun_out/r05zh_ab.txt
  env $cfg GMR_PHASE_TIMES=1 timeout -k 10 200 python -u bench.py --model diffmm --no-legs --no-cpu-baseline --no-probe --steps 5 --warmup 1 2>gpurun_out/r05zh_err.txt | cut -c1-200 >> gpurun_out/r05zh_ab.txt || exit $?
  grep phases gpurun_out/r05zh_err.txt | tail -2 >> gpurun_out/r05zh_ab.txt
done
