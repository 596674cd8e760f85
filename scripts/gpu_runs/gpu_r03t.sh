#!/bin/bash
# round 3: split-bf16 GEMM tile grouping (GMR_GEMM_GROUP) on the rebuild products: time and FETCH_SIZE
cd /root/repo
export TMPDIR=/tmp
for g in 0 4 8 16; do
  GMR_GEMM_GROUP=$g timeout -k 10 200 python -u scripts/gemm_bench.py --tiles 0 --mfma 6 --reps 10 --only "psample_h19k,psample_out19k,psample_post,train_out" > gpurun_out/r03t_group$g.txt 2>&1 || exit $?
  GMR_GEMM_GROUP=$g timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r03t_pmc$g -o pmc -- python3 scripts/gemm_bench.py --tiles 0 --mfma 6 --reps 3 --only "psample_h19k,psample_out19k,psample_post,train_out" > gpurun_out/r03t_pmc$g.log 2>&1 || exit $?
done
