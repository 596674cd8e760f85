#!/bin/bash
# fp16 scoring: kernel + GenRecV1 tests, then GenRecV1 bench lines with fp32 and fp16 scoring.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_genrec_gpu.py -k "score_f16 or rec_step_loss" -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/s16_tests.log 2>&1 || { tail -30 gpurun_out/s16_tests.log; exit 1; }
tail -1 gpurun_out/s16_tests.log
for d in fp32 fp16; do
  timeout -k 10 300 python bench.py --model genrecv1 --steps 2 --warmup 1 --no-cpu-baseline --scoring-dtype $d > gpurun_out/s16_bench_$d.json 2> gpurun_out/s16_bench_$d.err || { tail -20 gpurun_out/s16_bench_$d.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/s16_bench_$d.json'));print('$d', d['value'], d['eval_users_per_s'], d['eval_recall@20'], d['eval_scoring_dtype'])"
done
