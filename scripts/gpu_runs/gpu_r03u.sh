#!/bin/bash
# round 3: fused eval without LDS atomics (ballot slots): parity, timing, SQ counters of the kernel
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_score_topk_gpu.py tests/test_baby_gpu.py > gpurun_out/r03u_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/eval_profile.py --fused 1 > gpurun_out/r03u_eval.txt 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03u_prof -o prof -- python3 scripts/eval_profile.py --fused 1 --passes 20 > gpurun_out/r03u_prof.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d gpurun_out/r03u_pmc -o pmc -- python3 scripts/eval_profile.py --fused 1 --passes 3 > gpurun_out/r03u_pmc.log 2>&1
for g in 0 8; do
  GMR_GEMM_GROUP=$g timeout -k 10 200 python -u scripts/gemm_bench.py --tiles 0 --mfma 6 --reps 10 --only "psample_h19k,psample_out19k,psample_post,train_out" > gpurun_out/r03t_group$g.txt 2>&1 || exit $?
  GMR_GEMM_GROUP=$g timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r03t_pmc$g -o pmc -- python3 scripts/gemm_bench.py --tiles 0 --mfma 6 --reps 3 --only "psample_h19k,psample_out19k,psample_post,train_out" > gpurun_out/r03t_pmc$g.log 2>&1 || exit $?
done
