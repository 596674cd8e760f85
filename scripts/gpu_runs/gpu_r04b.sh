#!/bin/bash
# r04b: SpMM probe (what bounds the side-split SpMM at baby shape), then the r04a tests.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python scripts/micro/dump_graph.py baby norm_adj /tmp/na.bin && python scripts/micro/dump_graph.py baby ui_top1 /tmp/ui.bin || exit 1
timeout -k 10 120 scripts/micro/spmm_probe /tmp/na.bin > gpurun_out/r04b_probe.txt 2>&1 || { cat gpurun_out/r04b_probe.txt; exit 1; }
timeout -k 10 120 scripts/micro/spmm_probe /tmp/ui.bin >> gpurun_out/r04b_probe.txt 2>&1 || { cat gpurun_out/r04b_probe.txt; exit 1; }
cat gpurun_out/r04b_probe.txt
bash scripts/gpu_runs/gpu_r04a.sh
