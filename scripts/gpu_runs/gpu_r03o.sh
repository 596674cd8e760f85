#!/bin/bash
# round 3: side-split SpMM per-side times (both sides), small task sizes
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/spmm_side_balance.py > gpurun_out/r03o_balance.txt 2>&1 || exit $?
timeout -k 10 600 python -u scripts/spmm_side_sweep.py --Ts 8,12,16 --wpx 64,128,256 --tws 16,32 > gpurun_out/r03o_sweep.txt 2>&1
