#!/bin/bash
# round 5 (w): kernel trace of the GenRecV1 leg (current build): per-kernel totals per epoch, GPU-busy share
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05w_trace -o tr -- python3 -u bench.py --model genrecv1 --scoring-dtype fp16 --no-cpu-baseline --no-probe --steps 3 --warmup 1 > gpurun_out/r05w_trace.log 2>&1 || exit $?
