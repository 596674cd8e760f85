#!/bin/bash
# round 3: split-bf16 accuracy tests after the med3 clamp, DiffRec baby, then the default bench
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_diffrec_baby_gpu.py -k "x6 or diffrec_baby or side" > gpurun_out/r03d_tests.log 2>&1 || exit $?
GMR_PROBE_REPORT=1 timeout -k 10 900 python -u bench.py > gpurun_out/r03d_bench.json 2> gpurun_out/r03d_bench.err
