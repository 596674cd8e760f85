#!/bin/bash
# Quick check: the GPU tests of the given files, then the DiffMM bench with phases and probe.
set -o pipefail
TAG=${1:-quick}; shift
FILES=${@:-tests/test_kernels_gpu.py tests/test_diffmm_gpu.py}
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
timeout -k 10 400 python -u -m pytest $FILES -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread -q > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_tests.log; grep -E "FAILED|ERROR" gpurun_out/${TAG}_tests.log | head; fatal $rc tests
GMR_PHASE_TIMES=1 GMR_PROBE_REPORT=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-legs > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err; rc=$?
python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench.json'));print(d['value'], d['ms_per_step'], {k:v['frac'] for k,v in d['roofline_by_kernel'].items() if 'frac' in v})"; grep phases gpurun_out/${TAG}_bench.err | tr '\n' ' '; echo; grep -A3 "infonce:" gpurun_out/${TAG}_bench.err; fatal $rc bench
echo all-done
