#!/bin/bash
# round 5 (l): native graph executor - bit-exactness tests, epoch A/B (eager / hipGraphLaunch / executor)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_graph_capture_gpu.py \
  tests/test_resume_gpu.py > gpurun_out/r05l_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/r05l_tests.log
[ $rc -ne 0 ] && exit $rc
for cfg in "GMR_GRAPHS=0" "GMR_GRAPHS=1 GMR_GRAPH_EXEC=0" "GMR_GRAPHS=1" "GMR_GRAPHS=1 GMR_GRAPH_STREAMS=3" "GMR_GRAPHS=0" "GMR_GRAPHS=1"; do
  echo "=== $cfg" >> gpurun_out/r05l_ab.txt
  env $cfg GMR_PHASE_TIMES=1 timeout -k 10 200 python -u bench.py --model diffmm --no-legs --no-cpu-baseline --no-probe --steps 5 --warmup 1 2>gpurun_out/r05l_err.txt | cut -c1-200 >> gpurun_out/r05l_ab.txt || exit $?
  grep phases gpurun_out/r05l_err.txt | tail -2 >> gpurun_out/r05l_ab.txt
done
