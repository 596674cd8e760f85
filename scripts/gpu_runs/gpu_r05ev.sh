#!/bin/bash
# round-5 evidence on the current library: full GPU suite, smoke, serial rocprof summary of the bench
# epoch, PMC passes for the DiffMM, GenRecV1 and DiffRec workloads (stamped to this library, copied into profiles/ so the
# bench line and its legs carry their traffic), default bench line (with the DiffRec / GenRecV1 legs).
# usage: bash scripts/gpu_runs/gpu_r04ev.sh <tag>
set -o pipefail
TAG=${1:-r05ev}
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { case $1 in 0) ;; *) echo "fatal exit $1 in $2"; tail -20 gpurun_out/${TAG}_$2.log 2>/dev/null; exit 1;; esac; }
timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
echo "tests rc=$rc" >> gpurun_out/${TAG}_tests.log; tail -2 gpurun_out/${TAG}_tests.log; fatal $rc tests
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1; fatal $? smoke
GMR_SERIAL=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o prof -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-legs --no-probe > gpurun_out/${TAG}_prof.log 2>&1; fatal $? prof
for m in diffmm genrecv1 diffrec; do
  bash scripts/pmc_collect.sh $TAG $m > gpurun_out/${TAG}_pmc_$m.log 2>&1; fatal $? pmc_$m
  cp gpurun_out/${TAG}_pmc_$m.json profiles/
done
GMR_PROBE_REPORT=1 timeout -k 10 700 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err; fatal $? bench
cut -c1-400 gpurun_out/${TAG}_bench.json
echo all-done
