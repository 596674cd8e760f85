#!/bin/bash
# rocprofv3 passes over the SpMM microbenchmark: kernel durations, L2 hit/miss, HBM fetch.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
A="--segs ${SEGS:-128,32} --reps 20"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sp_kt -o kt -- python3 scripts/spmm_bench.py $A > gpurun_out/sp_kt.log 2>&1 &&
timeout -k 10 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/sp_pmc1 -o pmc -- python3 scripts/spmm_bench.py $A > gpurun_out/sp_pmc1.log 2>&1 &&
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/sp_pmc2 -o pmc -- python3 scripts/spmm_bench.py $A > gpurun_out/sp_pmc2.log 2>&1 &&
echo prof-done
