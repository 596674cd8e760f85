#!/bin/bash
# round 3: time-embedding backward parallel over h (diffusion tests), side-split SpMM per-side balance
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_diffmm_gpu.py tests/test_diffrec_gpu.py tests/test_phases_gpu.py > gpurun_out/r03n_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/spmm_side_balance.py > gpurun_out/r03n_balance.txt 2>&1 || exit $?
timeout -k 10 600 python -u scripts/spmm_side_sweep.py --Ts 16,32,64 --wpx 128,256,512 --tws 32 > gpurun_out/r03n_sweep.txt 2>&1
