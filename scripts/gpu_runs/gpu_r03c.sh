#!/bin/bash
# round 3: full GPU suite + default bench of the current tree
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 1500 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests > gpurun_out/r03c_tests.log 2>&1
echo "tests rc=$?" >> gpurun_out/r03c_tests.log
timeout -k 10 900 python -u bench.py > gpurun_out/r03c_bench.json 2> gpurun_out/r03c_bench.err
