#!/bin/bash
# round 6 (f): gc-row error diagnostics, the GPU suite after pruning, and an A/B of the BPR phase on a
# high-priority main stream (GMR_MAIN_PRIO)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q -s --timeout 200 --timeout-method thread tests/test_diffmm_train_gpu.py -m gpu \
  -k "diffusion_step_vs" > gpurun_out/r06f_gc.log 2>&1
grep -E "^\[|passed|failed" gpurun_out/r06f_gc.log
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu -k "not diffusion_step" \
  > gpurun_out/r06f_tests.log 2>&1 || { tail -60 gpurun_out/r06f_tests.log; exit 1; }
tail -2 gpurun_out/r06f_tests.log
for p in 0 1 0 1; do
  echo "=== GMR_MAIN_PRIO=$p" >> gpurun_out/r06f_ab.txt
  GMR_MAIN_PRIO=$p GMR_PHASE_TIMES=1 timeout -k 10 200 python -u bench.py --model diffmm --no-legs --no-cpu-baseline --no-probe --steps 5 --warmup 1 2>gpurun_out/r06f_err.txt | cut -c1-200 >> gpurun_out/r06f_ab.txt || exit $?
  grep phases gpurun_out/r06f_err.txt | tail -3 >> gpurun_out/r06f_ab.txt
done
cat gpurun_out/r06f_ab.txt
echo done
