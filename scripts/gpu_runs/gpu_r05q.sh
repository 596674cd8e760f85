#!/bin/bash
# round 5 (q): kernel trace of GenRecV1 phases (GPU-busy union per phase, launch counts)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05q_trace -o tr -- python3 -u scripts/phase_host_probe.py --model genrecv1 --reps 1 > gpurun_out/r05q_trace.log 2>&1 || exit $?
