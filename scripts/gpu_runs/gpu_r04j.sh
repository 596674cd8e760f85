#!/bin/bash
# r04j: pipelined split-bf16 InfoNCE (GMR_CL_PIPE): bit-exactness and fp64 tests, then the microbenchmark
# with the pipeline off / on.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py -k "contrast" > gpurun_out/r04j_tests.log 2>&1 || { tail -30 gpurun_out/r04j_tests.log; exit 1; }
tail -2 gpurun_out/r04j_tests.log
GMR_CL_PIPE=0 timeout -k 10 120 python scripts/contrast_bench.py > gpurun_out/r04j_bench.txt 2>&1 || { cat gpurun_out/r04j_bench.txt; exit 1; }
GMR_CL_PIPE=1 timeout -k 10 120 python scripts/contrast_bench.py >> gpurun_out/r04j_bench.txt 2>&1 || { cat gpurun_out/r04j_bench.txt; exit 1; }
cat gpurun_out/r04j_bench.txt
# A/B of the round-4 defaults on the bench epoch (phase wall times): the pre-split rebuild products
# (GMR_P3), the degree-class SpMM plan (GMR_SPMM_DC), the pipelined InfoNCE (GMR_CL_PIPE)
for v in "" "GMR_P3=0" "GMR_SPMM_DC=0" "GMR_CL_PIPE=0"; do
  env $v GMR_PHASE_TIMES=1 timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-legs --no-cpu-baseline --no-probe > gpurun_out/r04j_ab.json 2> gpurun_out/r04j_ab.err || { tail -20 gpurun_out/r04j_ab.err; exit 1; }
  echo "[$v] $(cut -c1-200 gpurun_out/r04j_ab.json | grep -o '"value": [0-9.]*, "unit": "users/s", "n_gpus": 1, "steps": 3, "warmup": 1, "ms_per_step": [0-9.]*')" >> gpurun_out/r04j_ab.txt
  grep 'phases' gpurun_out/r04j_ab.err | tail -3 >> gpurun_out/r04j_ab.txt
done
cat gpurun_out/r04j_ab.txt
