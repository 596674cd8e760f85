#!/bin/bash
# SQ stall counters over the SpMM microbenchmark (two --pmc passes, kernel-trace only).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
A="--segs ${SEGS:-128,32} --reps 10"
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES --output-format csv -d gpurun_out/sq1 -o pmc -- python3 scripts/spmm_bench.py $A > gpurun_out/sq1.log 2>&1 &&
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/sq2 -o pmc -- python3 scripts/spmm_bench.py $A > gpurun_out/sq2.log 2>&1 &&
echo sq-done
