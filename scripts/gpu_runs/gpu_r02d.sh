#!/bin/bash
# Full GPU test suite, SpMM plans on the baby graphs (incl. a collapsed-top-1 UI graph), and the
# DiffMM bench with phase times.
set -o pipefail
TAG=${1:-r02d}
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
timeout -k 10 600 python -u -m pytest tests -v -m gpu -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_tests.log; grep -E "FAILED|ERROR" gpurun_out/${TAG}_tests.log | head -20; fatal $rc tests
timeout -k 10 300 python scripts/spmm_bench.py --segs 65568,196640 --nbs 1,2,4 --reps 50 > gpurun_out/${TAG}_spmm.txt 2>&1; rc=$?
grep -v amdgpu gpurun_out/${TAG}_spmm.txt; fatal $rc spmm
GMR_PHASE_TIMES=1 GMR_PROBE_REPORT=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-legs > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err; rc=$?
head -c 400 gpurun_out/${TAG}_bench.json; echo; grep -A6 "spmm:" gpurun_out/${TAG}_bench.err; fatal $rc bench
echo all-done
