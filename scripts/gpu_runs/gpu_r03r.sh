#!/bin/bash
# round 3: full GPU suite + default bench of the current tree
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r03r_tests.log 2>&1
echo "tests rc=$?" >> gpurun_out/r03r_tests.log
GMR_PROBE_REPORT=1 timeout -k 10 600 python -u bench.py > gpurun_out/r03r_bench.json 2> gpurun_out/r03r_bench.err
