#!/bin/bash
# r04o: fused GenRecV1 decoder stack (gmr_decoder_*): fused vs layer-by-layer tests, the GenRecV1 suites,
# then the GenRecV1 bench with the per-class probe (launch counts and times).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 250 --timeout-method thread -p no:cacheprovider \
  tests/test_decoder_gpu.py tests/test_genrec_gpu.py tests/test_genrec_tiktok_gpu.py tests/test_tiktok_gpu.py tests/test_dist_gpu.py tests/test_kernels_gpu.py -k "decoder or genrec or tiktok or GenRec or denoiser or contrast or dp2" > gpurun_out/r04o_tests.log 2>&1 || { tail -50 gpurun_out/r04o_tests.log; exit 1; }
tail -3 gpurun_out/r04o_tests.log
GMR_PROBE_REPORT=1 timeout -k 10 300 python bench.py --model genrecv1 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r04o_bench.json 2> gpurun_out/r04o_bench.err || { tail -30 gpurun_out/r04o_bench.err; exit 1; }
cut -c1-300 gpurun_out/r04o_bench.json; grep -E "^---|launches" gpurun_out/r04o_bench.err | head -20
GMR_DEC_FUSED=0 timeout -k 10 300 python bench.py --model genrecv1 --steps 3 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/r04o_bench_unfused.json 2> gpurun_out/r04o_bench_unfused.err || { tail -30 gpurun_out/r04o_bench_unfused.err; exit 1; }
cut -c1-300 gpurun_out/r04o_bench_unfused.json
