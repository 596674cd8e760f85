#!/bin/bash
# Round-end check: smoke(), the GenRecV1 and sports-shaped bench lines (the DiffMM baby line and
# the parity suite come from scripts/gpu_round.sh).
set -o pipefail
TAG=${1:-fin}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -30 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 500 python bench.py --model genrecv1 --steps 2 --warmup 1 > gpurun_out/${TAG}_genrec_bench.json 2> gpurun_out/${TAG}_genrec_bench.err || { tail -30 gpurun_out/${TAG}_genrec_bench.err; exit 1; }
cut -c1-300 gpurun_out/${TAG}_genrec_bench.json
timeout -k 10 500 python bench.py --shape sports --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_sports_bench.json 2> gpurun_out/${TAG}_sports_bench.err || { tail -30 gpurun_out/${TAG}_sports_bench.err; exit 1; }
cut -c1-300 gpurun_out/${TAG}_sports_bench.json
echo all-done
