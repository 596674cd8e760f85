#!/bin/bash
# Memory-side traffic and MFMA busy cycles per kernel class of one bench workload, on the current
# build.  Three separate rocprofv3 --pmc passes (FETCH_SIZE and WRITE_SIZE do not fit one pass on
# gfx950; MFMA busy + GRBM active in a third), each over the same short serial bench command, then
# scripts/pmc_summary.py writes gpurun_out/<tag>_pmc_<model>.json stamped with the library's SHA-256
# (bench.py uses a summary only when that hash equals the loaded library's).
# usage: scripts/pmc_collect.sh <tag> <model> [extra bench args]
set -o pipefail
TAG=${1:-dev}; MODEL=${2:-diffmm}; shift 2
export TMPDIR=/tmp
mkdir -p gpurun_out
CMD="bench.py --model $MODEL --steps 1 --warmup 1 --no-cpu-baseline --no-probe --no-legs --eval-passes 1 $*"
export GMR_SERIAL=1
timeout -k 10 -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_pmcf_${MODEL} -o pmc -- python3 $CMD > gpurun_out/${TAG}_pmcf_${MODEL}.log 2>&1 || { echo "fetch pass failed"; tail -20 gpurun_out/${TAG}_pmcf_${MODEL}.log; exit 1; }
timeout -k 10 -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_pmcw_${MODEL} -o pmc -- python3 $CMD > gpurun_out/${TAG}_pmcw_${MODEL}.log 2>&1 || { echo "write pass failed"; tail -20 gpurun_out/${TAG}_pmcw_${MODEL}.log; exit 1; }
timeout -k 10 -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${TAG}_pmcm_${MODEL} -o pmc -- python3 $CMD > gpurun_out/${TAG}_pmcm_${MODEL}.log 2>&1 || { echo "mfma pass failed"; tail -20 gpurun_out/${TAG}_pmcm_${MODEL}.log; exit 1; }
python3 scripts/pmc_summary.py gpurun_out/${TAG}_pmcf_${MODEL}/pmc_counter_collection.csv gpurun_out/${TAG}_pmcw_${MODEL}/pmc_counter_collection.csv gpurun_out/${TAG}_pmcm_${MODEL}/pmc_counter_collection.csv "$CMD" > gpurun_out/${TAG}_pmc_${MODEL}.json && cat gpurun_out/${TAG}_pmc_${MODEL}.json
