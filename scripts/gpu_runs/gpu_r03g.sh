#!/bin/bash
# round 3: serial rocprofv3 kernel summary + PMC passes for the headline and both legs, on this build
set -o pipefail
TAG=${1:-r03g}
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { case $1 in 0) ;; *) echo "fatal exit $1 in $2"; exit 1;; esac; }
GMR_SERIAL=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o prof -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-legs --no-probe > gpurun_out/${TAG}_prof.log 2>&1; fatal $? rocprof
bash scripts/pmc_collect.sh $TAG diffmm > /dev/null; fatal $? pmc_diffmm
bash scripts/pmc_collect.sh $TAG diffrec > /dev/null; fatal $? pmc_diffrec
bash scripts/pmc_collect.sh $TAG genrecv1 > /dev/null; fatal $? pmc_genrecv1
echo all-done
