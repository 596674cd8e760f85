#!/bin/bash
# Round-2 check: GPU parity tests (incl. the 2-rank DP test), GEMM tile/split sweep of the
# long-K denoiser shapes, the default bench, and a serial-mode rocprof kernel summary.
# A failing test does not stop the measurements; a crash, abort or time-out stops everything.
set -o pipefail
TAG=${1:-r02a}
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
timeout -k 10 600 python -u -m pytest tests -v -m gpu -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
tail -3 gpurun_out/${TAG}_tests.log; grep -E "FAILED|ERROR" gpurun_out/${TAG}_tests.log | head; fatal $rc tests
timeout -k 10 300 python scripts/gemm_bench.py --only "train_h,dh (NN),train_out,dW2,dW1,psample_h (NT),psample_out (NT)" --tiles 64,128,256,256128,128256 --splits 1,2,4,8 --reps 10 > gpurun_out/${TAG}_gemm.txt 2>&1; rc=$?; fatal $rc gemm
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err; rc=$?
cat gpurun_out/${TAG}_bench.json; fatal $rc bench
GMR_SERIAL=1 timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o prof -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/${TAG}_prof.log 2>&1; rc=$?; fatal $rc rocprof
echo all-done
