#!/bin/bash
# Round-2 verification on one MI355X: the full -m gpu suite, the default bench line (headline +
# legs + cpu baseline), the serial rocprofv3 kernel summary and the PMC passes on this build.
set -o pipefail
TAG=${1:-r02z}
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
timeout -k 10 600 python -u -m pytest tests -v -m gpu -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_tests.log; grep -E "FAILED|ERROR" gpurun_out/${TAG}_tests.log | head -20; fatal $rc tests
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err; rc=$?
head -c 1500 gpurun_out/${TAG}_bench.json; echo; tail -3 gpurun_out/${TAG}_bench.err; fatal $rc bench
GMR_SERIAL=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o prof -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-legs --no-probe > gpurun_out/${TAG}_prof.log 2>&1; rc=$?; fatal $rc rocprof
bash scripts/pmc_collect.sh $TAG diffmm; rc=$?; fatal $rc pmc
echo all-done
