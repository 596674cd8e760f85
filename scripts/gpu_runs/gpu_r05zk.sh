#!/bin/bash
# round 5 (zk): InfoNCE grid targets re-swept in the epoch (GMR_CL_WG_ROWS x GMR_CL_WG_TABLE) on the current step order
set -o pipefail
mkdir -p gpurun_out
for r in 512 384 768; do for t in 768 512 1024; do
  echo "=== rows $r table $t" >> gpurun_out/r05zk_ab.txt
  GMR_CL_WG_ROWS=$r GMR_CL_WG_TABLE=$t GMR_PHASE_TIMES=1 timeout -k 10 200 python -u bench.py --model diffmm --no-legs --no-cpu-baseline --no-probe --steps 4 --warmup 1 2>gpurun_out/r05zk_err.txt | cut -c1-200 >> gpurun_out/r05zk_ab.txt || exit $?
  grep phases gpurun_out/r05zk_err.txt | tail -1 >> gpurun_out/r05zk_ab.txt
done; done
