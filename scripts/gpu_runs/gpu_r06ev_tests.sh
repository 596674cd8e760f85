#!/bin/bash
# round-6 evidence, part 1: the full GPU suite and smoke() on the current library
# usage: bash scripts/gpu_runs/gpu_r06ev_tests.sh <tag>
set -o pipefail
TAG=${1:-r06ev}
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { case $1 in 0) ;; *) echo "fatal exit $1 in $2"; tail -30 gpurun_out/${TAG}_$2.log 2>/dev/null; exit 1;; esac; }
sha256sum generative-multimodal-recommendation_amd/gmr/libgmr_hip.so | tee gpurun_out/${TAG}_lib_sha.txt
timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
echo "tests rc=$rc" >> gpurun_out/${TAG}_tests.log; tail -2 gpurun_out/${TAG}_tests.log; fatal $rc tests
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1; fatal $? smoke
tail -2 gpurun_out/${TAG}_smoke.log
echo all-done
