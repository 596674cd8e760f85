#!/bin/bash
# A/B of environment knobs on the DiffMM bench (same box, back to back; the first setting is run
# again at the end to show the box's drift).  usage: scripts/gpu_env_ab.sh TAG "ENV1" "ENV2" ...
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
i=0
for KN in "$@" "$1"; do
i=$((i+1))
env $KN GMR_PHASE_TIMES=1 GMR_PROBE_REPORT=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-legs > gpurun_out/${TAG}_b$i.json 2> gpurun_out/${TAG}_b$i.err; rc=$?
echo "== [$KN]"; python -c "import json;d=json.load(open('gpurun_out/${TAG}_b$i.json'));print(d['value'], d['ms_per_step'], {k:v['frac'] for k,v in d['roofline_by_kernel'].items() if 'frac' in v})"; grep phases gpurun_out/${TAG}_b$i.err | tail -1; grep -A1 -E "^--- (spmm|gemm)" gpurun_out/${TAG}_b$i.err | grep -- "---"; fatal $rc bench
done
echo all-done
