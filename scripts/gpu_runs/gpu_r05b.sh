#!/bin/bash
# round 5 (b): baby-shape parity tests + the folded p_sample chain's tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -v --timeout 400 --timeout-method thread \
  tests/test_psample_fold_gpu.py tests/test_diffmm_baby_train_gpu.py tests/test_vbpr_baby_gpu.py \
  tests/test_kmeans_tiktok_gpu.py tests/test_score_topk_gpu.py \
  tests/test_kernels_gpu.py::test_spmm_side_all_hub_rows_split_blocks tests/test_kernels_gpu.py::test_split3_planes_exact \
  tests/test_baby_gpu.py::test_p_sample_top1_all_users tests/test_diffrec_baby_gpu.py tests/test_diffmm_gpu.py \
  tests/test_diffrec_gpu.py tests/test_sports_gpu.py tests/test_phases_gpu.py \
  > gpurun_out/r05b_tests.log 2>&1
echo "tests rc=$?" >> gpurun_out/r05b_tests.log
