#!/bin/bash
# r04e: the pre-split GEMM kernel tests, then the round-4 parity tests (fused eval at baby / sports, quick_start, DP, GenRecV1 tiny + TikTok).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py -k "p3 or split3 or x6" > gpurun_out/r04e_p3tests.log 2>&1 || { tail -30 gpurun_out/r04e_p3tests.log; exit 1; }
tail -3 gpurun_out/r04e_p3tests.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 420 --timeout-method thread -p no:cacheprovider -s \
  tests/test_score_topk_gpu.py tests/test_baby_gpu.py tests/test_sports_gpu.py tests/test_quick_start_gpu.py \
  tests/test_dist_gpu.py tests/test_genrec_gpu.py tests/test_genrec_tiktok_gpu.py > gpurun_out/r04e_tests.log 2>&1
rc=$?
tail -25 gpurun_out/r04e_tests.log
exit $rc
