#!/bin/bash
# round 5 (y): kernel timeline of the current DiffMM rec step (steps queued behind a GPU blocker)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05y_trace -o tr -- python3 -u scripts/host_vs_gpu_probe.py --steps 5 > gpurun_out/r05y_trace.log 2>&1 || exit $?
