#!/bin/bash
# round 3: InfoNCE split-bf16 passes: grid-size sweep (workgroups per rows / table pass)
cd /root/repo
export TMPDIR=/tmp
: > gpurun_out/r03y_cl_sweep.txt
for ra in 256 512 1024 2048; do
  for tb in 384 768 1536 3072; do
    echo "== rows $ra table $tb" >> gpurun_out/r03y_cl_sweep.txt
    GMR_CL_WG_ROWS=$ra GMR_CL_WG_TABLE=$tb timeout -k 10 120 python -u scripts/contrast_bench.py --reps 20 >> gpurun_out/r03y_cl_sweep.txt 2>&1 || exit $?
  done
done
