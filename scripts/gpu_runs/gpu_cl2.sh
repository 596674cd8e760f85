#!/bin/bash
# K8 InfoNCE after the finalize/reduce changes: microbench (+ per-kernel rocprof) and parity tests.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python scripts/contrast_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cl2_prof -o prof -- python3 scripts/contrast_bench.py > gpurun_out/cl2_prof.log 2>&1 || { tail -20 gpurun_out/cl2_prof.log; exit 1; }
python3 - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/cl2_prof/prof_kernel_stats.csv')):
    if 'cl_' in r['Name']:
        print(r['Name'].split('(')[0][-40:], r['Calls'], round(float(r['AverageNs'])/1e3, 1), 'us avg')
PY
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "diffmm or contrast or genrec" > gpurun_out/cl2_tests.log 2>&1 || { tail -30 gpurun_out/cl2_tests.log; exit 1; }
tail -1 gpurun_out/cl2_tests.log
