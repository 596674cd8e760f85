#!/bin/bash
# round 3: side-split SpMM launch-shape sweep + the DP tests
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 600 python -u scripts/spmm_side_sweep.py --reps 50 > gpurun_out/r03b_sweep.txt 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_dist_gpu.py > gpurun_out/r03b_dist.log 2>&1
