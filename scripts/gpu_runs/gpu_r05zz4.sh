#!/bin/bash
# round 5 (zz4): LDS bank-conflict and MFMA pass over the GenRecV1 and DiffRec legs (serial streams)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp GMR_SERIAL=1
for m in genrecv1 diffrec; do
  timeout -k 10 -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/r05zz4_$m -o pmc -- python3 bench.py --model $m --steps 1 --warmup 1 --no-cpu-baseline --no-probe --no-legs --eval-passes 1 > gpurun_out/r05zz4_$m.log 2>&1 || exit 1
done
