#!/bin/bash
# round 5 (c): the full GPU suite (VBPR now pinned to the fp64 reference run)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests/ > gpurun_out/r05c_tests.log 2>&1
echo "tests rc=$?" >> gpurun_out/r05c_tests.log
GMR_PROBE_REPORT=1 timeout -k 10 300 python -u bench.py --model diffmm --no-legs --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r05c_bench.json 2> gpurun_out/r05c_probe.txt
