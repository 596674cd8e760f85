#!/bin/bash
# round 5 (zf): the DP path on RCCL with one rank (tests/test_rccl_gpu.py)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_rccl_gpu.py > gpurun_out/r05zf_tests.log 2>&1 || exit $?
