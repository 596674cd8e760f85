#!/bin/bash
# r04a: the eval-path parity tests (fused default + GMR_EVAL_FUSED=0) at baby / sports, the tightened
# fused-vs-unfused float test, the quick_start / main.py entry tests, the DP tests.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 420 --timeout-method thread -p no:cacheprovider -s \
  tests/test_score_topk_gpu.py tests/test_baby_gpu.py tests/test_sports_gpu.py tests/test_quick_start_gpu.py \
  tests/test_dist_gpu.py tests/test_genrec_gpu.py > gpurun_out/r04a_tests.log 2>&1
rc=$?
tail -25 gpurun_out/r04a_tests.log
exit $rc
