#!/bin/bash
# round 3: rehearsal of the driver's multi-GPU leg on one GPU: bench.py --gpus 2 launches its own two
# ranks (gloo instead of RCCL: two ranks cannot share one GPU under RCCL), headline + legs + dp_local
cd /root/repo
export TMPDIR=/tmp
GMR_DIST_BACKEND=gloo timeout -k 10 900 python -u bench.py --gpus 2 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r03x_dp2.json 2> gpurun_out/r03x_dp2.err
