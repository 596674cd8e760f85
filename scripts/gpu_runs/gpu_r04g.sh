#!/bin/bash
# r04g: DiffMM epoch with the rec step replayed from a HIP graph (GMR_GRAPHS=1) vs eager, alternating, 5 steps
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in a b c; do
  for g in 0 1; do
    GMR_GRAPHS=$g timeout -k 10 300 python bench.py --model diffmm --no-legs --steps 5 --warmup 2 --no-cpu-baseline --no-probe > gpurun_out/r04g_g${g}_$r.json 2> gpurun_out/r04g_g${g}_$r.err || { tail -20 gpurun_out/r04g_g${g}_$r.err; exit 1; }
    echo "GMR_GRAPHS=$g ($r) $(python -c "import json; d=json.load(open('gpurun_out/r04g_g${g}_$r.json')); print(d['value'], d['ms_per_step'], d['eval_recall@20'])")"
  done
done | tee gpurun_out/r04g_ab.txt
