#!/bin/bash
# round 3: side-split SpMM parity + A/B against the lane plans, the new DP / accuracy tests
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "side or x6" > gpurun_out/r03a_tests.log 2>&1
rc=$?
echo "kernel tests rc=$rc" >> gpurun_out/r03a_tests.log
[ $rc -ne 0 ] && exit $rc
for s in 0 1; do
  GMR_SPMM_SIDE=$s timeout -k 10 200 python scripts/spmm_bench.py --segs 65568 --graphs norm_adj,ui_top1,ui_hub --reps 100 > gpurun_out/r03a_spmm_side$s.txt 2>&1 || exit $?
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_dist_gpu.py > gpurun_out/r03a_dist.log 2>&1
