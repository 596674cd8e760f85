#!/bin/bash
# round 3: side-split SpMM entries-in-flight (EB 8 vs 16) x workgroups per XCD at T = 16
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 600 python -u scripts/spmm_side_sweep.py --Ts 16 --wpx 128,256,512 --tws 32 --ebs 8,16 > gpurun_out/r03eb_sweep.txt 2>&1
