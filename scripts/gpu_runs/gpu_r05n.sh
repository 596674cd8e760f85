#!/bin/bash
# round 5 (n): graph capture without the allocator-cache flush; per-step eager / hipGraph / executor probe; epoch A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_graph_capture_gpu.py \
  > gpurun_out/r05n_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/graph_step_probe.py --steps 50 > gpurun_out/r05n_probe.txt 2>&1 || exit $?
for cfg in "GMR_GRAPHS=0" "GMR_GRAPHS=1 GMR_GRAPH_EXEC=0" "GMR_GRAPHS=1" "GMR_GRAPHS=0" "GMR_GRAPHS=1"; do
  echo "=== $cfg" >> gpurun_out/r05n_ab.txt
  env $cfg GMR_PHASE_TIMES=1 timeout -k 10 200 python -u bench.py --model diffmm --no-legs --no-cpu-baseline --no-probe --steps 5 --warmup 1 2>gpurun_out/r05n_err.txt | cut -c1-200 >> gpurun_out/r05n_ab.txt || exit $?
  grep phases gpurun_out/r05n_err.txt | tail -2 >> gpurun_out/r05n_ab.txt
done
timeout -k 10 400 python -u scripts/dp_shard_probe.py --worlds 1,2,4,8 --epochs 3 > gpurun_out/r05n_dp_global.txt 2>&1 || exit $?
timeout -k 10 400 python -u scripts/dp_shard_probe.py --worlds 2,4,8 --epochs 3 --mode local > gpurun_out/r05n_dp_local.txt 2>&1 || exit $?
