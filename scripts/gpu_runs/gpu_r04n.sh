#!/bin/bash
# r04n: fused eval with item quarters per row block (shared thresholds, in-workgroup merge); DiffMM
# modality projections on the split kernel (GMR_PROJ_X6).  Kernel + reference parity tests, the eval
# microbenchmark, and the headline epoch A/B with phase times.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 250 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py::test_contrast_pipelined_bit_exact tests/test_kernels_gpu.py::test_contrast_table_fixup_bit_exact tests/test_kernels_gpu.py::test_contrast_fused_vs_fp64 tests/test_score_topk_gpu.py tests/test_baby_gpu.py tests/test_sports_gpu.py tests/test_diffmm_gpu.py tests/test_phases_gpu.py tests/test_genrec_tiktok_gpu.py > gpurun_out/r04n_tests.log 2>&1 || { tail -40 gpurun_out/r04n_tests.log; exit 1; }
tail -3 gpurun_out/r04n_tests.log
GMR_EVAL_X6=0 timeout -k 10 120 python scripts/score_topk_bench.py > gpurun_out/r04n_topk.txt 2>&1 || { cat gpurun_out/r04n_topk.txt; exit 1; }
GMR_EVAL_X6=1 timeout -k 10 120 python scripts/score_topk_bench.py >> gpurun_out/r04n_topk.txt 2>&1 || { cat gpurun_out/r04n_topk.txt; exit 1; }
cat gpurun_out/r04n_topk.txt
for v in "GMR_PROJ_X6=1" "GMR_PROJ_X6=0"; do
  env $v GMR_PHASE_TIMES=1 timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-legs --no-cpu-baseline --no-probe > gpurun_out/r04n_ab.json 2> gpurun_out/r04n_ab.err || { tail -20 gpurun_out/r04n_ab.err; exit 1; }
  echo "[$v] $(cut -c1-250 gpurun_out/r04n_ab.json | grep -o '"value": [0-9.]*, "unit": "users/s", "n_gpus": 1, "steps": 3, "warmup": 1, "ms_per_step": [0-9.]*')" >> gpurun_out/r04n_ab.txt
  grep -E 'phases|eval' gpurun_out/r04n_ab.err | tail -4 >> gpurun_out/r04n_ab.txt
  grep -o '"eval_users_per_s": [0-9.]*' gpurun_out/r04n_ab.json >> gpurun_out/r04n_ab.txt || true
done
cat gpurun_out/r04n_ab.txt
