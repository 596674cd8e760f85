#!/bin/bash
# Bench lines for the other BASELINE configs on one GPU: GenRecV1 TikTok-shaped (config 5, with a
# rocprofv3 kernel summary) and DiffMM Amazon-sports-shaped (config 4's per-GPU workload at N=1).
set -o pipefail
TAG=${1:-cfg}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python bench.py --model genrecv1 --steps 2 --warmup 1 > gpurun_out/${TAG}_genrec_bench.json 2> gpurun_out/${TAG}_genrec_bench.err || { echo "genrec bench failed"; tail -30 gpurun_out/${TAG}_genrec_bench.err; exit 1; }
cat gpurun_out/${TAG}_genrec_bench.json
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_genrec_prof -o prof -- python3 bench.py --model genrecv1 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_genrec_prof.log 2>&1 || { echo "genrec rocprof failed"; tail -30 gpurun_out/${TAG}_genrec_prof.log; exit 1; }
timeout -k 10 500 python bench.py --shape sports --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_sports_bench.json 2> gpurun_out/${TAG}_sports_bench.err || { echo "sports bench failed"; tail -30 gpurun_out/${TAG}_sports_bench.err; exit 1; }
cat gpurun_out/${TAG}_sports_bench.json
echo all-done
