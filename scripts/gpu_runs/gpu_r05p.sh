#!/bin/bash
# round 5 (p): host-bound or GPU-bound per phase (GenRecV1 TikTok, DiffMM baby)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/phase_host_probe.py --model genrecv1 > gpurun_out/r05p_genrec.txt 2>&1 || exit $?
timeout -k 10 300 python -u scripts/phase_host_probe.py --model diffmm > gpurun_out/r05p_diffmm.txt 2>&1 || exit $?
