#!/bin/bash
# round 5 (zq): 128 x 64 tiles for the N = 64 NN projections: epoch A/B against the library without them
# (ablibs/libgmr_base.so: the same objects with the previous gemm.hip), DiffMM and VBPR-free legs
set -o pipefail
mkdir -p gpurun_out
for lib in base new base new; do
  if [ $lib = base ]; then L=ablibs/libgmr_base.so; else L=generative-multimodal-recommendation_amd/gmr/libgmr_hip.so; fi
  echo "=== $lib" >> gpurun_out/r05zq_ab.txt
  GMR_HIP_LIB=$L GMR_PHASE_TIMES=1 timeout -k 10 200 python -u bench.py --model diffmm --no-legs --no-cpu-baseline --no-probe --steps 5 --warmup 1 2>gpurun_out/r05zq_err.txt | cut -c1-200 >> gpurun_out/r05zq_ab.txt || exit $?
  grep phases gpurun_out/r05zq_err.txt | tail -2 >> gpurun_out/r05zq_ab.txt
done
