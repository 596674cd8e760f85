#!/bin/bash
# SpMM lane/packed plans at 8 vs 16 gathers per lane-group batch (GMR_SPMM_EB).
set -o pipefail
TAG=${1:-eb}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k spmm -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
GMR_SPMM_EB=16 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k spmm -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests16.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests16.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests16.log
for eb in 8 16; do
  echo "== GMR_SPMM_EB=$eb"
  GMR_SPMM_EB=$eb GMR_SPMM_WPX_PACKED=512 timeout -k 10 200 python scripts/spmm_bench.py --segs 65568,196640 > gpurun_out/${TAG}_bench_eb$eb.txt 2>&1 || { tail -20 gpurun_out/${TAG}_bench_eb$eb.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/${TAG}_bench_eb$eb.txt
done
