#!/bin/bash
# round 5 (zm): fused-eval float-embedding test with the principled tie bound
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_score_topk_gpu.py > gpurun_out/r05zm_tests.log 2>&1 || exit $?
