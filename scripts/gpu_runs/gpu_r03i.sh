#!/bin/bash
# round 3: where the eval pass goes (fused vs unfused), kernel trace of the fused passes
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/eval_profile.py --fused 0 > gpurun_out/r03i_eval.txt 2>&1 || exit $?
timeout -k 10 300 python -u scripts/eval_profile.py --fused 1 >> gpurun_out/r03i_eval.txt 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03i_prof -o prof -- python3 scripts/eval_profile.py --fused 1 --passes 20 > gpurun_out/r03i_prof.log 2>&1
