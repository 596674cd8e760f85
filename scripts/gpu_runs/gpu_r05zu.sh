#!/bin/bash
# round 5 (zu): same-box epoch A/B of the final library against the round's evidence-3 GEMM objects
# (ablibs/libgmr_r05ev3.so: gemm.hip / gemm_x6.hip of c8df4f7 linked with the current other objects)
set -o pipefail
mkdir -p gpurun_out
for lib in ev3 new ev3 new ev3 new; do
  if [ $lib = ev3 ]; then L=ablibs/libgmr_r05ev3.so; else L=generative-multimodal-recommendation_amd/gmr/libgmr_hip.so; fi
  echo "=== $lib" >> gpurun_out/r05zu_ab.txt
  GMR_HIP_LIB=$L GMR_PHASE_TIMES=1 timeout -k 10 200 python -u bench.py --model diffmm --no-legs --no-cpu-baseline --no-probe --steps 5 --warmup 1 2>gpurun_out/r05zu_err.txt | cut -c1-200 >> gpurun_out/r05zu_ab.txt || exit $?
  grep phases gpurun_out/r05zu_err.txt | tail -2 >> gpurun_out/r05zu_ab.txt
done
