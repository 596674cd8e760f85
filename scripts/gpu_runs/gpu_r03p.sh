#!/bin/bash
# round 3: side-split SpMM with DPP group broadcasts instead of LDS shuffles: DPP semantics check, SpMM
# parity tests, per-graph timings
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 60 ./scripts/micro/dpp_bcast_test > gpurun_out/r03p_dpp.txt 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "spmm or side or bipartite or csr" > gpurun_out/r03p_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/spmm_side_balance.py > gpurun_out/r03p_balance.txt 2>&1 || exit $?
timeout -k 10 600 python -u scripts/spmm_side_sweep.py --Ts 12,16,32 --wpx 128,256 --tws 32 > gpurun_out/r03p_sweep.txt 2>&1
