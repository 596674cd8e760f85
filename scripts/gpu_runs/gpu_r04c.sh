#!/bin/bash
# r04c: side-SpMM isolation probe (plan parts switched off, scripts/micro/side_iso.cpp), then the
# pre-split GEMM prototype (scripts/micro/p3_micro.hip), the round-4 parity tests (r04a set) after the fused-vs-unfused tie-window change.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python scripts/micro/dump_graph.py baby norm_adj /tmp/na.bin > gpurun_out/r04c_probe.txt || exit 1
timeout -k 10 180 scripts/micro/side_iso /tmp/na.bin >> gpurun_out/r04c_probe.txt 2>&1 || { cat gpurun_out/r04c_probe.txt; exit 1; }
timeout -k 10 180 scripts/micro/p3_micro > gpurun_out/r04c_p3.txt 2>&1 || { cat gpurun_out/r04c_p3.txt; exit 1; }
cat gpurun_out/r04c_p3.txt
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py -k "p3 or split3 or x6" > gpurun_out/r04c_p3tests.log 2>&1 || { tail -30 gpurun_out/r04c_p3tests.log; exit 1; }
tail -3 gpurun_out/r04c_p3tests.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 420 --timeout-method thread -p no:cacheprovider -s \
  tests/test_score_topk_gpu.py tests/test_baby_gpu.py tests/test_sports_gpu.py tests/test_quick_start_gpu.py \
  tests/test_dist_gpu.py tests/test_genrec_gpu.py tests/test_genrec_tiktok_gpu.py > gpurun_out/r04c_tests.log 2>&1
rc=$?
tail -25 gpurun_out/r04c_tests.log
exit $rc
