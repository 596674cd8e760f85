#!/bin/bash
# round 6 (b): stream-ordering guards + host tape; A/B of the tape on the DiffMM epoch (alternating, same box)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_stream_order_gpu.py \
  tests/test_diffmm_gpu.py tests/test_phases_gpu.py tests/test_resume_gpu.py tests/test_graph_capture_gpu.py -m gpu \
  > gpurun_out/r06b_tests.log 2>&1 || { tail -40 gpurun_out/r06b_tests.log; exit 1; }
tail -2 gpurun_out/r06b_tests.log
for t in 0 1 0 1 0 1; do
  echo "=== GMR_TAPE=$t" >> gpurun_out/r06b_ab.txt
  GMR_TAPE=$t GMR_PHASE_TIMES=1 timeout -k 10 200 python -u bench.py --model diffmm --no-legs --no-cpu-baseline --no-probe --steps 5 --warmup 1 2>gpurun_out/r06b_err.txt | cut -c1-200 >> gpurun_out/r06b_ab.txt || exit $?
  grep phases gpurun_out/r06b_err.txt | tail -3 >> gpurun_out/r06b_ab.txt
done
cat gpurun_out/r06b_ab.txt
