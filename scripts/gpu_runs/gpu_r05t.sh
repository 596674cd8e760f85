#!/bin/bash
# round 5 (t): host-overhead cuts (gemm call plans, cached slab views): GenRecV1 + DiffMM epochs, host profile
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 200 python -u bench.py --model genrecv1 --scoring-dtype fp16 --no-cpu-baseline --no-probe --steps 5 --warmup 1 2>>gpurun_out/r05t_err.txt | cut -c1-240 >> gpurun_out/r05t_ab.txt || exit $?
timeout -k 10 200 python -u bench.py --model diffmm --no-legs --no-cpu-baseline --no-probe --steps 5 --warmup 1 2>>gpurun_out/r05t_err.txt | cut -c1-240 >> gpurun_out/r05t_ab.txt || exit $?
done
timeout -k 10 300 python -u scripts/host_profile.py --model genrecv1 > gpurun_out/r05t_hostprof.txt 2>&1 || exit $?
