#!/bin/bash
# Multi-job SpMM launches: their GPU tests, then the DiffMM bench with and without them (A/B).
set -o pipefail
TAG=${1:-r02g}
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_diffmm_gpu.py tests/test_phases_gpu.py tests/test_baby_gpu.py -v -m gpu -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_tests.log; grep -E "FAILED|ERROR" gpurun_out/${TAG}_tests.log | head -20; fatal $rc tests
for F in ${FUSES:-0 1 9 11 7}; do
GMR_SPMM_FUSE=$F GMR_PHASE_TIMES=1 GMR_PROBE_REPORT=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-legs > gpurun_out/${TAG}_bench_f$F.json 2> gpurun_out/${TAG}_bench_f$F.err; rc=$?
echo "== fuse $F"; head -c 300 gpurun_out/${TAG}_bench_f$F.json; echo; grep -A12 "spmm:" gpurun_out/${TAG}_bench_f$F.err; grep phases gpurun_out/${TAG}_bench_f$F.err | tail -1; fatal $rc bench
done
echo all-done
