#!/bin/bash
# A/B of tuning knobs on the DiffMM bench: rebuild chunk, InfoNCE workgroup targets.
set -o pipefail
TAG=${1:-r02m}
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_diffmm_gpu.py -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread -q > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_tests.log; grep -E "FAILED|ERROR" gpurun_out/${TAG}_tests.log | head; fatal $rc tests
i=0
for KN in "" "GMR_REBUILD_CHUNK=19456" "GMR_CL_WG_ROWS=1024 GMR_CL_WG_TABLE=1536" "GMR_CL_WG_ROWS=2048 GMR_CL_WG_TABLE=2048" ""; do
i=$((i+1))
env $KN GMR_PHASE_TIMES=1 GMR_PROBE_REPORT=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-legs > gpurun_out/${TAG}_b$i.json 2> gpurun_out/${TAG}_b$i.err; rc=$?
echo "== [$KN]"; python -c "import json;d=json.load(open('gpurun_out/${TAG}_b$i.json'));print(d['value'], d['ms_per_step'])"; grep phases gpurun_out/${TAG}_b$i.err | tr '\n' ' '; echo; grep -A3 "infonce:" gpurun_out/${TAG}_b$i.err; fatal $rc bench
done
echo all-done
