#!/bin/bash
# GenRecV1 GPU parity tests, verbose log under gpurun_out/.  usage: gpu_genrec.sh TAG [pytest -k expr]
set -o pipefail
TAG=${1:-gr}
K=${2:-}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_genrec_gpu.py ${K:+-k "$K"} -m gpu -v --tb=short --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/${TAG}_tests.log | tail -40
exit $rc
