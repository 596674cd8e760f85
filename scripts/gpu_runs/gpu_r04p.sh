#!/bin/bash
# r04p: the fused-decoder checks (r04o), then the round's evidence on the same library (r04ev2).
set -o pipefail
bash scripts/gpu_runs/gpu_r04o.sh && bash scripts/gpu_runs/gpu_r04ev.sh r04ev2
