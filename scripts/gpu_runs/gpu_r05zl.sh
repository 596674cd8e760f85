#!/bin/bash
# round 5 (zl): split-K slab minimum of the split-bf16 plans re-swept in the epoch (GMR_X6_MIN_SLAB)
set -o pipefail
mkdir -p gpurun_out
for v in default 1024 256 default 1024 256; do
  echo "=== min_slab $v" >> gpurun_out/r05zl_ab.txt
  if [ $v = default ]; then E=""; else E="GMR_X6_MIN_SLAB=$v"; fi
  env $E GMR_PHASE_TIMES=1 timeout -k 10 200 python -u bench.py --model diffmm --no-legs --no-cpu-baseline --no-probe --steps 4 --warmup 1 2>gpurun_out/r05zl_err.txt | cut -c1-200 >> gpurun_out/r05zl_ab.txt || exit $?
  grep phases gpurun_out/r05zl_err.txt | tail -1 >> gpurun_out/r05zl_ab.txt
done
