#!/bin/bash
# HBM traffic of the bench workload per kernel class: two separate rocprofv3 --pmc passes
# (FETCH_SIZE and WRITE_SIZE do not fit one pass on gfx950), then scripts/pmc_traffic.py.
# usage: scripts/pmc_traffic.sh <tag> [bench args...]   (e.g. --model genrecv1, --shape sports)
set -o pipefail
TAG=${1:-dev}; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_pmc_fetch -o pmc -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-probe "$@" > gpurun_out/${TAG}_pmc_fetch.log 2>&1 || { echo "fetch pass failed"; tail -20 gpurun_out/${TAG}_pmc_fetch.log; exit 1; }
timeout -k 10 500 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_pmc_write -o pmc -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-probe "$@" > gpurun_out/${TAG}_pmc_write.log 2>&1 || { echo "write pass failed"; tail -20 gpurun_out/${TAG}_pmc_write.log; exit 1; }
python3 scripts/pmc_traffic.py gpurun_out/${TAG}_pmc_fetch/pmc_counter_collection.csv gpurun_out/${TAG}_pmc_write/pmc_counter_collection.csv > gpurun_out/${TAG}_pmc_traffic.json && cat gpurun_out/${TAG}_pmc_traffic.json
