#!/bin/bash
# round 3: fused score -> mask -> top-k eval kernel: parity tests, the eval-using model tests, bench
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_score_topk_gpu.py tests/test_baby_gpu.py tests/test_sports_gpu.py tests/test_vbpr_gpu.py tests/test_genrec_gpu.py tests/test_eval_extras.py tests/test_diffmm_gpu.py > gpurun_out/r03h_tests.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/r03h_bench.json 2> gpurun_out/r03h_bench.err
