#!/bin/bash
# round 5 (a): new baby-shape parity tests, the folded p_sample chain, the SpMM relabel probe, a DiffMM bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread \
  tests/test_psample_fold_gpu.py tests/test_diffmm_baby_train_gpu.py tests/test_vbpr_baby_gpu.py \
  tests/test_kmeans_tiktok_gpu.py tests/test_score_topk_gpu.py \
  tests/test_kernels_gpu.py::test_spmm_side_all_hub_rows_split_blocks tests/test_kernels_gpu.py::test_split3_planes_exact \
  tests/test_baby_gpu.py::test_p_sample_top1_all_users tests/test_diffrec_baby_gpu.py tests/test_diffmm_gpu.py \
  > gpurun_out/r05a_tests.log 2>&1
rc=$?
echo "tests rc=$rc" >> gpurun_out/r05a_tests.log
[ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -ge 128 ] && exit $rc
timeout -k 10 200 python -u scripts/spmm_relabel_probe.py > gpurun_out/r05a_relabel.txt 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --model diffmm --no-legs --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/r05a_bench.json 2> gpurun_out/r05a_bench.err
