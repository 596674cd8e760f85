#!/bin/bash
# round-6 evidence, part 2: serial rocprof summary of the bench epoch and the PMC passes for the DiffMM,
# GenRecV1 and DiffRec workloads (stamped to this library, copied into profiles/)
# usage: bash scripts/gpu_runs/gpu_r06ev_perf.sh <tag>
set -o pipefail
TAG=${1:-r06ev}
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { case $1 in 0) ;; *) echo "fatal exit $1 in $2"; tail -20 gpurun_out/${TAG}_$2.log 2>/dev/null; exit 1;; esac; }
sha256sum generative-multimodal-recommendation_amd/gmr/libgmr_hip.so | tee gpurun_out/${TAG}_lib_sha.txt
GMR_SERIAL=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o prof -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-legs --no-probe > gpurun_out/${TAG}_prof.log 2>&1; fatal $? prof
for m in diffmm genrecv1 diffrec; do
  bash scripts/pmc_collect.sh $TAG $m > gpurun_out/${TAG}_pmc_$m.log 2>&1; fatal $? pmc_$m
  cp gpurun_out/${TAG}_pmc_$m.json profiles/
done
echo all-done
