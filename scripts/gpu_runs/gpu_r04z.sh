#!/bin/bash
# r04z: GMR_GEMM_STAGES64 2 (default) vs 3 on the GenRecV1 and DiffMM epochs, three alternating rounds, 5 steps
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in a b c; do
  for s in 2 3; do
    for m in genrecv1 diffmm; do
      GMR_GEMM_STAGES64=$s timeout -k 10 300 python bench.py --model $m --no-legs --steps 5 --warmup 2 --no-cpu-baseline --no-probe > gpurun_out/r04z_${m}_s${s}_$r.json 2> gpurun_out/r04z_${m}_s${s}_$r.err || { tail -20 gpurun_out/r04z_${m}_s${s}_$r.err; exit 1; }
      echo "$m STAGES64=$s ($r) $(python -c "import json; d=json.load(open('gpurun_out/r04z_${m}_s${s}_$r.json')); print(d['value'], d['ms_per_step'])")"
    done
  done
done | tee gpurun_out/r04z_ab.txt
