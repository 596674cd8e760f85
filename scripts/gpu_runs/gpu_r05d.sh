#!/bin/bash
# round 5 (d): VBPR baby tests; serial-epoch kernel stats of the folded-chain build
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_vbpr_baby_gpu.py > gpurun_out/r05d_tests.log 2>&1
echo "tests rc=$?" >> gpurun_out/r05d_tests.log
GMR_SERIAL=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05d_prof -o prof -- python3 bench.py --model diffmm --steps 2 --warmup 1 --no-cpu-baseline --no-legs --no-probe > gpurun_out/r05d_prof.log 2>&1
echo "prof rc=$?" >> gpurun_out/r05d_prof.log
