#!/bin/bash
# round 5 (f): rec-step tests after the assemble-overwrite change; default bench line with legs + phase times
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_diffmm_gpu.py \
  tests/test_diffmm_baby_train_gpu.py tests/test_phases_gpu.py tests/test_sports_gpu.py tests/test_dist_gpu.py \
  tests/test_resume_gpu.py tests/test_graph_capture_gpu.py > gpurun_out/r05f_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/r05f_tests.log
[ $rc -ge 124 ] && exit $rc
GMR_PHASE_TIMES=1 timeout -k 10 900 python -u bench.py > gpurun_out/r05f_bench.json 2> gpurun_out/r05f_bench.err
