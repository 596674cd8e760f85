#!/bin/bash
# round 6 (c): rec-step fusions (bpr+sqnorm, loss+mw+acc, clear-after-read instead of fills, scatter+nbwd,
# table reduce+nbwd, assemble+nbwd, split-K reduce+leaky+normalize): full GPU suite, then the epoch x3
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu \
  > gpurun_out/r06c_tests.log 2>&1 || { tail -60 gpurun_out/r06c_tests.log; exit 1; }
tail -2 gpurun_out/r06c_tests.log
for t in 1 2 3; do
  GMR_PHASE_TIMES=1 timeout -k 10 200 python -u bench.py --model diffmm --no-legs --no-cpu-baseline --no-probe --steps 5 --warmup 1 2>gpurun_out/r06c_err.txt | cut -c1-200 >> gpurun_out/r06c_ab.txt || exit $?
  grep phases gpurun_out/r06c_err.txt | tail -3 >> gpurun_out/r06c_ab.txt
done
cat gpurun_out/r06c_ab.txt
