#!/bin/bash
# GPU tests (new: D10 edge drop, sampler properties, resume), the default bench with its legs,
# the serial rocprof kernel summary and the PMC passes (traffic + MFMA busy) of the DiffMM workload.
set -o pipefail
TAG=${1:-r02c}
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
timeout -k 10 600 python -u -m pytest tests -v -m gpu -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_tests.log; grep -E "FAILED|ERROR" gpurun_out/${TAG}_tests.log | head; fatal $rc tests
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err; rc=$?
cat gpurun_out/${TAG}_bench.json | head -c 3000; echo; tail -5 gpurun_out/${TAG}_bench.err; fatal $rc bench
GMR_SERIAL=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o prof -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-legs --no-probe > gpurun_out/${TAG}_prof.log 2>&1; rc=$?; fatal $rc rocprof
bash scripts/pmc_collect.sh $TAG diffmm; rc=$?; fatal $rc pmc
echo all-done
