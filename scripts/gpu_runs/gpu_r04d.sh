#!/bin/bash
# r04d: SpMM row-end store probe (scripts/micro/spmm_probe.hip V5-V8), the pre-split GEMM kernel tests,
# then the round-4 parity tests (fused eval at baby / sports, quick_start, DP, GenRecV1 tiny + TikTok).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python scripts/micro/dump_graph.py baby norm_adj /tmp/na.bin > gpurun_out/r04d_probe.txt || exit 1
timeout -k 10 120 scripts/micro/spmm_probe /tmp/na.bin >> gpurun_out/r04d_probe.txt 2>&1 || { cat gpurun_out/r04d_probe.txt; exit 1; }
grep -E 'V2|V5|V6|V7|V8' gpurun_out/r04d_probe.txt
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py -k "p3 or split3 or x6" > gpurun_out/r04d_p3tests.log 2>&1 || { tail -30 gpurun_out/r04d_p3tests.log; exit 1; }
tail -3 gpurun_out/r04d_p3tests.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 420 --timeout-method thread -p no:cacheprovider -s \
  tests/test_score_topk_gpu.py tests/test_baby_gpu.py tests/test_sports_gpu.py tests/test_quick_start_gpu.py \
  tests/test_dist_gpu.py tests/test_genrec_gpu.py tests/test_genrec_tiktok_gpu.py > gpurun_out/r04d_tests.log 2>&1
rc=$?
tail -25 gpurun_out/r04d_tests.log
exit $rc
