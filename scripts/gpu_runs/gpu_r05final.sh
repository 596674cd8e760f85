#!/bin/bash
# round 5 final check on the committed tree: full GPU suite + smoke
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r05final_tests.log 2>&1; rc=$?
echo "tests rc=$rc" >> gpurun_out/r05final_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05final_smoke.log 2>&1
