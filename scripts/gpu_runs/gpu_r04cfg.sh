#!/bin/bash
# r04cfg: per-config bench lines on the final library: DiffMM sports-shaped (config 4's per-GPU workload, with
# its serial probe for the section-6 projection), GenRecV1 TikTok-shaped with fp16 scoring (config 5), DiffRec baby.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
GMR_PROBE_REPORT=1 timeout -k 10 600 python bench.py --model diffmm --shape sports --no-legs --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r04cfg_sports.json 2> gpurun_out/r04cfg_sports.err || { tail -20 gpurun_out/r04cfg_sports.err; exit 1; }
cut -c1-200 gpurun_out/r04cfg_sports.json
timeout -k 10 300 python bench.py --model genrecv1 --scoring-dtype fp16 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r04cfg_genrec16.json 2> gpurun_out/r04cfg_genrec16.err || { tail -20 gpurun_out/r04cfg_genrec16.err; exit 1; }
cut -c1-200 gpurun_out/r04cfg_genrec16.json
timeout -k 10 300 python bench.py --model diffrec --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r04cfg_diffrec.json 2> gpurun_out/r04cfg_diffrec.err || { tail -20 gpurun_out/r04cfg_diffrec.err; exit 1; }
cut -c1-200 gpurun_out/r04cfg_diffrec.json
