#!/bin/bash
# r04y: GenRecV1 epoch A/B (alternating, two rounds): default | GMR_X6_MIN_SLAB=128 | GMR_GEMM_STAGES64=3
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
G="python bench.py --model genrecv1 --steps 3 --warmup 1 --no-cpu-baseline --no-probe"
for r in a b; do
  for cfg in "DEF=1" "GMR_X6_MIN_SLAB=128" "GMR_GEMM_STAGES64=3"; do
    t=$(echo $cfg | tr '=' '_')
    env $cfg timeout -k 10 300 $G > gpurun_out/r04y_${t}_$r.json 2> gpurun_out/r04y_${t}_$r.err || { tail -20 gpurun_out/r04y_${t}_$r.err; exit 1; }
    echo "$cfg ($r) $(python -c "import json; d=json.load(open('gpurun_out/r04y_${t}_$r.json')); print(d['value'], d['ms_per_step'])")"
  done
done | tee gpurun_out/r04y_ab.txt
