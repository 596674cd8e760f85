#!/bin/bash
# round 5 (r): host synchronisations inside the GenRecV1 epoch phases
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/sync_probe.py --model genrecv1 > gpurun_out/r05r_sync.txt 2>&1 || exit $?
