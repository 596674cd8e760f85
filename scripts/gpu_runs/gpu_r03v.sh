#!/bin/bash
# round 3 final build: full GPU suite, default bench, serial rocprof summary, PMC passes (stamped)
set -o pipefail
TAG=${1:-r03v}
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { case $1 in 0) ;; *) echo "fatal exit $1 in $2"; exit 1;; esac; }
timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
echo "tests rc=$rc" >> gpurun_out/${TAG}_tests.log; fatal $rc tests
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1; fatal $? smoke
GMR_SERIAL=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o prof -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-legs --no-probe > gpurun_out/${TAG}_prof.log 2>&1; fatal $? rocprof
bash scripts/pmc_collect.sh $TAG diffmm > /dev/null; fatal $? pmc_diffmm
bash scripts/pmc_collect.sh $TAG diffrec > /dev/null; fatal $? pmc_diffrec
bash scripts/pmc_collect.sh $TAG genrecv1 > /dev/null; fatal $? pmc_genrecv1
echo all-done
