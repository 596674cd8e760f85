#!/bin/bash
# round 3: early E0 all-reduce (DP tests), eval pass profile fused vs unfused
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_dist_gpu.py tests/test_sports_gpu.py -k "dp" > gpurun_out/r03j_dist.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/eval_profile.py --fused 0 > gpurun_out/r03j_eval.txt 2>&1 || exit $?
timeout -k 10 300 python -u scripts/eval_profile.py --fused 1 >> gpurun_out/r03j_eval.txt 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03j_prof -o prof -- python3 scripts/eval_profile.py --fused 1 --passes 20 > gpurun_out/r03j_prof.log 2>&1
timeout -k 10 300 python -u scripts/gemm_bench.py --tiles 64 --mfma 32,6 --acc --only "tf_,proj,cl_,train_Z,dout" > gpurun_out/r03j_gemm64.txt 2>&1
timeout -k 10 300 python -u scripts/gemm_bench.py --tiles 128,256128 --mfma 6 --only "train_,psample_h19k,psample_out19k" > gpurun_out/r03j_gemm_x6tiles.txt 2>&1
