#!/bin/bash
# GPU-box check used during development: parity tests, a short bench, a rocprofv3 kernel summary.
# usage: scripts/gpu_check.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-dev}; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests -q -m gpu -p no:cacheprovider -x > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 400 python bench.py --steps 2 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o prof -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/${TAG}_prof.log 2>&1 || { echo "rocprof failed"; tail -30 gpurun_out/${TAG}_prof.log; exit 1; }
echo done
