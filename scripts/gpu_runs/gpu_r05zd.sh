#!/bin/bash
# round 5 (zd): DiffMM rebuild with the image graph built beside the text sweep: tests, epoch phases
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_diffmm_gpu.py \
  tests/test_resume_gpu.py tests/test_phases_gpu.py tests/test_baby_gpu.py tests/test_dist_gpu.py tests/test_graph_capture_gpu.py \
  > gpurun_out/r05zd_tests.log 2>&1 || exit $?
for i in 1 2 3; do
  GMR_PHASE_TIMES=1 timeout -k 10 200 python -u bench.py --model diffmm --no-legs --no-cpu-baseline --no-probe --steps 5 --warmup 1 2>gpurun_out/r05zd_err.txt | cut -c1-200 >> gpurun_out/r05zd_ab.txt || exit $?
  grep phases gpurun_out/r05zd_err.txt | tail -2 >> gpurun_out/r05zd_ab.txt
done
