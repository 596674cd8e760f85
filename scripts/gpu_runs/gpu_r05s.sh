#!/bin/bash
# round 5 (s): host profile of a GenRecV1 epoch (cProfile)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/host_profile.py --model genrecv1 > gpurun_out/r05s_hostprof.txt 2>&1 || exit $?
