#!/bin/bash
# r04sw: existing split-bf16 GEMM switches re-measured on the final library's DiffMM epoch (two alternating rounds)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python bench.py --model diffmm --no-legs --steps 5 --warmup 2 --no-cpu-baseline --no-probe"
for r in a b; do
  for cfg in "DEF=1" "GMR_GEMM_X6_PIPE=1" "GMR_GEMM_X6_NB128=1" "GMR_GEMM_X6_NB128=2" "GMR_GEMM_X6_NB128=3"; do
    t=$(echo $cfg | tr '=' '_')
    env $cfg timeout -k 10 300 $B > gpurun_out/r04sw_${t}_$r.json 2> gpurun_out/r04sw_${t}_$r.err || { tail -20 gpurun_out/r04sw_${t}_$r.err; exit 1; }
    echo "$cfg ($r) $(python -c "import json; d=json.load(open('gpurun_out/r04sw_${t}_$r.json')); print(d['value'], d['ms_per_step'])")"
  done
done | tee gpurun_out/r04sw_ab.txt
