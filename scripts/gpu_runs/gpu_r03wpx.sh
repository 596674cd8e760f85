#!/bin/bash
# round 3: side SpMM at 128 workgroups per XCD for d = 256 too: SpMM / model tests, default bench
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_diffmm_gpu.py tests/test_baby_gpu.py tests/test_phases_gpu.py -k "spmm or side or forward or rec_step or baby or phase" > gpurun_out/r03wpx_tests.log 2>&1 || exit $?
GMR_PROBE_REPORT=1 timeout -k 10 700 python -u bench.py > gpurun_out/r03wpx_bench.json 2> gpurun_out/r03wpx_bench.err
