#!/bin/bash
# Packed lane-plan SpMM: parity tests, then the microbenchmark against the lane plan at several
# workgroups-per-XCD caps of the packed kernel.
set -o pipefail
TAG=${1:-pk}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k spmm -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
for w in ${WPXS:-64 128 256 512}; do
  echo "== GMR_SPMM_WPX_PACKED=$w"
  GMR_SPMM_WPX_PACKED=$w timeout -k 10 200 python scripts/spmm_bench.py --segs 65568,196640 > gpurun_out/${TAG}_bench_w$w.txt 2>&1 || { tail -20 gpurun_out/${TAG}_bench_w$w.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/${TAG}_bench_w$w.txt
done
