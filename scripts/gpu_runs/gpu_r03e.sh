#!/bin/bash
# round 3: split-bf16 InfoNCE parity + A/B in the bench epoch
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_diffmm_gpu.py tests/test_phases_gpu.py -k "contrast or rec_step or phase or forward" > gpurun_out/r03e_tests.log 2>&1 || exit $?
timeout -k 10 900 python -u bench.py --no-legs --no-cpu-baseline > gpurun_out/r03e_bench.json 2> gpurun_out/r03e_bench.err
