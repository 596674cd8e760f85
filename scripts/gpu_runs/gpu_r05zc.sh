#!/bin/bash
# round 5 (zc): GenRecV1 rebuild chunks over two vs three streams
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_genrec_gpu.py \
  tests/test_genrec_tiktok_gpu.py tests/test_decoder_gpu.py tests/test_dist_gpu.py tests/test_resume_gpu.py \
  > gpurun_out/r05zc_tests.log 2>&1 || exit $?
for cfg in "GMR_GR_REBUILD_STREAMS=2" "GMR_GR_REBUILD_STREAMS=3" "GMR_GR_REBUILD_STREAMS=2" "GMR_GR_REBUILD_STREAMS=3"; do
  echo "=== $cfg" >> gpurun_out/r05zc_ab.txt
  env $cfg timeout -k 10 200 python -u bench.py --model genrecv1 --scoring-dtype fp16 --no-cpu-baseline --no-probe --steps 5 --warmup 1 2>>gpurun_out/r05zc_err.txt | cut -c1-200 >> gpurun_out/r05zc_ab.txt || exit $?
done
for cfg in "GMR_GR_REBUILD_STREAMS=2" "GMR_GR_REBUILD_STREAMS=3"; do
  echo "=== $cfg" >> gpurun_out/r05zc_phases.txt
  env $cfg timeout -k 10 300 python -u scripts/phase_host_probe.py --model genrecv1 --reps 2 2>&1 | grep rep >> gpurun_out/r05zc_phases.txt || exit $?
done
