#!/bin/bash
# r04gap: kernel trace of the DiffMM bench with its side streams on (the timed configuration), for the idle-gap
# analysis of whole epochs (scripts/epoch_gaps.py)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04gap_prof -o run -- python3 bench.py --model diffmm --no-legs --steps 2 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/r04gap.log 2>&1 || { tail -20 gpurun_out/r04gap.log; exit 1; }
f=$(find gpurun_out/r04gap_prof -name "*kernel_trace.csv" | head -1); gzip -c "$f" > gpurun_out/r04gap_kernel_trace.csv.gz; ls -la gpurun_out/r04gap_kernel_trace.csv.gz
