#!/bin/bash
# round 5 (u): decoder layers issued from C++ - bit-identity tests, GenRecV1 parity suites, epoch A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_decoder_gpu.py \
  tests/test_genrec_gpu.py tests/test_genrec_tiktok_gpu.py > gpurun_out/r05u_tests.log 2>&1 || exit $?
for cfg in "GMR_DEC_NATIVE=0" "GMR_DEC_NATIVE=1" "GMR_DEC_NATIVE=0" "GMR_DEC_NATIVE=1"; do
  echo "=== $cfg" >> gpurun_out/r05u_ab.txt
  env $cfg timeout -k 10 200 python -u bench.py --model genrecv1 --scoring-dtype fp16 --no-cpu-baseline --no-probe --steps 5 --warmup 1 2>>gpurun_out/r05u_err.txt | cut -c1-200 >> gpurun_out/r05u_ab.txt || exit $?
done
timeout -k 10 500 python -u scripts/dp_shard_probe.py --shape sports --worlds 1,8 --epochs 2 > gpurun_out/r05u_dp_sports_global.txt 2>&1 || exit $?
timeout -k 10 300 python -u scripts/dp_shard_probe.py --shape sports --worlds 8 --epochs 2 --mode local > gpurun_out/r05u_dp_sports_local.txt 2>&1 || exit $?
