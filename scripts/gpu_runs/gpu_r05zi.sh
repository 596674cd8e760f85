#!/bin/bash
# round 5 (zi): GenRecV1 text branch of the rec step on a side stream (GMR_GR_MODAL_STREAMS): parity suites, A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_genrec_gpu.py \
  tests/test_genrec_tiktok_gpu.py tests/test_dist_gpu.py tests/test_resume_gpu.py > gpurun_out/r05zi_tests.log 2>&1 || exit $?
for cfg in "GMR_GR_MODAL_STREAMS=0" "GMR_GR_MODAL_STREAMS=1" "GMR_GR_MODAL_STREAMS=0" "GMR_GR_MODAL_STREAMS=1"; do
  echo "=== $cfg" >> gpurun_out/r05zi_ab.txt
  env $cfg timeout -k 10 200 python -u bench.py --model genrecv1 --scoring-dtype fp16 --no-cpu-baseline --no-probe --steps 5 --warmup 1 2>>gpurun_out/r05zi_err.txt | cut -c1-200 >> gpurun_out/r05zi_ab.txt || exit $?
done
