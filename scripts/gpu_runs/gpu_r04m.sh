#!/bin/bash
# r04m: GenRecV1 cross-attention as head tables (gmr_xattn_*) + table reuse across p_sample steps:
# GenRecV1 GPU tests (tiny goldens incl. dropout grads vs torch, TikTok fixture, DP), then the GenRecV1
# bench with the per-class probe (launch counts).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 250 --timeout-method thread -p no:cacheprovider \
  tests/test_genrec_gpu.py tests/test_genrec_tiktok_gpu.py tests/test_tiktok_gpu.py tests/test_dist_gpu.py -k "genrec or tiktok or GenRec or denoiser" > gpurun_out/r04m_tests.log 2>&1 || { tail -40 gpurun_out/r04m_tests.log; exit 1; }
tail -3 gpurun_out/r04m_tests.log
GMR_PROBE_REPORT=1 timeout -k 10 300 python bench.py --model genrecv1 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r04m_bench.json 2> gpurun_out/r04m_bench.err || { tail -30 gpurun_out/r04m_bench.err; exit 1; }
cut -c1-300 gpurun_out/r04m_bench.json; grep -E "^---|launches" gpurun_out/r04m_bench.err | head -20
