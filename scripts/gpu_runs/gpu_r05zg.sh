#!/bin/bash
# round 5 (zg): K2 alone before the InfoNCE fork, H after it (GMR_K2_FIRST): tests, A/B
set -o pipefail
mkdir -p gpurun_out
GMR_K2_FIRST=1 timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_diffmm_gpu.py \
  tests/test_graph_capture_gpu.py tests/test_diffmm_baby_train_gpu.py > gpurun_out/r05zg_tests.log 2>&1 || exit $?
for cfg in "GMR_K2_FIRST=0" "GMR_K2_FIRST=1" "GMR_K2_FIRST=0" "GMR_K2_FIRST=1" "GMR_K2_FIRST=0" "GMR_K2_FIRST=1"; do
  echo "=== $cfg" >> gpurun_out/r05zg_ab.txt
  env $cfg GMR_PHASE_TIMES=1 timeout -k 10 200 python -u bench.py --model diffmm --no-legs --no-cpu-baseline --no-probe --steps 5 --warmup 1 2>gpurun_out/r05zg_err.txt | cut -c1-200 >> gpurun_out/r05zg_ab.txt || exit $?
  grep phases gpurun_out/r05zg_err.txt | tail -2 >> gpurun_out/r05zg_ab.txt
done
