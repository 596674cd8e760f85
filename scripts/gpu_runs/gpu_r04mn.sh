#!/bin/bash
# r04m + r04n in one call (the pool is congested): GenRecV1 cross-attention tables + table reuse, the
# fused eval with item quarters, DiffMM projections on the split kernel.
set -o pipefail
bash scripts/gpu_runs/gpu_r04m.sh && bash scripts/gpu_runs/gpu_r04n.sh
