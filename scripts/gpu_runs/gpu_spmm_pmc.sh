#!/bin/bash
# SQ / TCC / TCP counters of the SpMM variants on norm_adj at d = 128 (one rocprofv3 --pmc pass each).
set -o pipefail
TAG=${1:-spmmpmc}
mkdir -p gpurun_out
export TMPDIR=/tmp
B="scripts/spmm_bench.py --segs 65568,196640,262144 --graphs norm_adj --nbs 2 --reps 5"
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_BUSY_CYCLES --output-format csv -d gpurun_out/${TAG}_sq -o pmc -- python3 $B > gpurun_out/${TAG}_sq.log 2>&1 || { echo "sq pass failed"; tail -5 gpurun_out/${TAG}_sq.log; exit 1; }
timeout -k 10 -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${TAG}_tcc -o pmc -- python3 $B > gpurun_out/${TAG}_tcc.log 2>&1 || { echo "tcc pass failed"; tail -5 gpurun_out/${TAG}_tcc.log; exit 1; }
echo all-done
