#!/bin/bash
# round 3: fused eval with pipelined prefetch + LDS-staged masks; 64^2 split tiles for NT calls
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_score_topk_gpu.py tests/test_kernels_gpu.py -k "score or topk or x6 or gemm" > gpurun_out/r03k_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/eval_profile.py --fused 1 > gpurun_out/r03k_eval.txt 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03k_prof -o prof -- python3 scripts/eval_profile.py --fused 1 --passes 20 > gpurun_out/r03k_prof.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_genrec_gpu.py tests/test_baby_gpu.py tests/test_tiktok_gpu.py > gpurun_out/r03k_tests2.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/r03k_bench.json 2> gpurun_out/r03k_bench.err
