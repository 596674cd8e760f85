#!/bin/bash
# Full round check: parity tests + bench + rocprof (gpu_check.sh), the default bench (with the
# CPU-baseline leg), and a 2-rank gloo data-parallel rehearsal on the single GPU.
set -o pipefail
TAG=${1:-dev}
export TMPDIR=/tmp
bash scripts/gpu_check.sh "$TAG" || exit 1
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench_default.json 2> gpurun_out/${TAG}_bench_default.err || { echo "default bench failed"; tail -30 gpurun_out/${TAG}_bench_default.err; exit 1; }
cat gpurun_out/${TAG}_bench_default.json
GMR_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_dp2.json 2> gpurun_out/${TAG}_dp2.err || { echo "dp2 failed"; tail -30 gpurun_out/${TAG}_dp2.err; exit 1; }
cat gpurun_out/${TAG}_dp2.json
echo all-done
