#!/bin/bash
# K8 InfoNCE: range-reduced expf vs v_exp_f32 (GMR_CL_FASTEXP=1): microbench + parity tests.
set -o pipefail
export TMPDIR=/tmp
for f in 0 1 0 1; do
  echo "== GMR_CL_FASTEXP=$f"
  GMR_CL_FASTEXP=$f timeout -k 10 120 python scripts/contrast_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
done
GMR_CL_FASTEXP=1 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "diffmm or contrast or genrec or infonce" > gpurun_out/clexp_tests.log 2>&1 || { tail -30 gpurun_out/clexp_tests.log; exit 1; }
tail -1 gpurun_out/clexp_tests.log
