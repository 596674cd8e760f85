#!/bin/bash
# SpMM lane plans at 4 vs 8 lanes per row (16- vs 32-column XCD slices).
set -o pipefail
export TMPDIR=/tmp
for l in 4 8; do
  echo "== GMR_SPMM_LPR=$l"
  GMR_SPMM_LPR=$l timeout -k 10 200 python scripts/spmm_bench.py --segs 65568,196640 > gpurun_out/lpr$l.txt 2>&1 || { tail -20 gpurun_out/lpr$l.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/lpr$l.txt
done
