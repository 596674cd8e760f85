#!/bin/bash
# round 5 (x): two k groups per 64^2 split-bf16 block (PIPE 3) vs the one-group ring (PIPE 2): GEMM timing, x6 tests, epoch A/B
set -o pipefail
mkdir -p gpurun_out
GMR_X6_RING=2 timeout -k 10 120 python -u scripts/x6_small_bench.py > gpurun_out/r05x_gemm.txt 2>&1 || exit $?
GMR_X6_RING=1 timeout -k 10 120 python -u scripts/x6_small_bench.py >> gpurun_out/r05x_gemm.txt 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "gemm or x6" \
  tests/test_decoder_gpu.py tests/test_genrec_gpu.py tests/test_genrec_tiktok_gpu.py > gpurun_out/r05x_tests.log 2>&1 || exit $?
for cfg in "GMR_X6_RING=2" "GMR_X6_RING=1" "GMR_X6_RING=2" "GMR_X6_RING=1"; do
  echo "=== $cfg" >> gpurun_out/r05x_ab.txt
  env $cfg timeout -k 10 200 python -u bench.py --model genrecv1 --scoring-dtype fp16 --no-cpu-baseline --no-probe --steps 5 --warmup 1 2>>gpurun_out/r05x_err.txt | cut -c1-200 >> gpurun_out/r05x_ab.txt || exit $?
  env $cfg timeout -k 10 200 python -u bench.py --model diffmm --no-legs --no-cpu-baseline --no-probe --steps 5 --warmup 1 2>>gpurun_out/r05x_err.txt | cut -c1-200 >> gpurun_out/r05x_ab.txt || exit $?
done
