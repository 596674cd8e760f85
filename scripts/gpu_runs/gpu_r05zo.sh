#!/bin/bash
# round 5 (zo): MFMA busy of the projection GEMM (one PMC pass over the single-shape benchmark)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/r05zo_pmc -o pmc -- python3 scripts/gemm_bench.py --only proj_v --tiles 64 --mfma 32 --splits 8 --reps 10 > gpurun_out/r05zo.log 2>&1 || exit $?
