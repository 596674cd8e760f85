#!/bin/bash
# SpMM development check: the SpMM kernel tests, then lane / packed / chunk plans on the
# baby-shaped DiffMM graphs (row-major and column-panel sources).
set -o pipefail
TAG=${1:-spmm}
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -v -m gpu -p no:cacheprovider -k "spmm" --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_tests.log; grep -E "FAILED|ERROR" gpurun_out/${TAG}_tests.log | head -20; fatal $rc tests
[ $rc -ne 0 ] && exit 1
timeout -k 10 300 python scripts/spmm_bench.py --segs 65568,196640,262144 --panel --reps 50 > gpurun_out/${TAG}_bench.txt 2>&1; rc=$?
cat gpurun_out/${TAG}_bench.txt; fatal $rc bench
echo all-done
