#!/bin/bash
# round 6 (s): per-kernel stall / LDS breakdown of the DiffMM epoch on the final build (serial streams), two SQ passes,
# as round 5 (zy): wave cycles split into parked (s_waitcnt / barrier), issue-stalled and issuing, and LDS bank
# conflicts per LDS-array cycle
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp GMR_SERIAL=1
CMD="bench.py --model diffmm --steps 1 --warmup 1 --no-cpu-baseline --no-probe --no-legs --eval-passes 1"
timeout -k 10 -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/r06s_a -o pmc -- python3 $CMD > gpurun_out/r06s_a.log 2>&1 || exit 1
timeout -k 10 -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/r06s_b -o pmc -- python3 $CMD > gpurun_out/r06s_b.log 2>&1 || exit 1
echo all-done
