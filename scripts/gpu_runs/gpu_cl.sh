#!/bin/bash
# K8 InfoNCE grid sweep (workgroups per pass).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for a in ${ROWS:-512 1024 2048}; do for b in ${TABS:-512 1024 2048}; do
  echo "== rows $a table $b"
  GMR_CL_WG_ROWS=$a GMR_CL_WG_TABLE=$b timeout -k 10 120 python scripts/contrast_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
done; done
