#!/bin/bash
# round 3: config 4's per-GPU workload (DiffMM sports-shaped) on the final build
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 900 python -u bench.py --shape sports --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03sp_sports.json 2> gpurun_out/r03sp_sports.err
