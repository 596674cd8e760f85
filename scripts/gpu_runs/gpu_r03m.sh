#!/bin/bash
# round 3: fused eval without LDS atomics (ballot slots): parity, timing, SQ counters of the kernel
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_score_topk_gpu.py tests/test_baby_gpu.py > gpurun_out/r03m_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/eval_profile.py --fused 1 > gpurun_out/r03m_eval.txt 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03m_prof -o prof -- python3 scripts/eval_profile.py --fused 1 --passes 20 > gpurun_out/r03m_prof.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d gpurun_out/r03m_pmc -o pmc -- python3 scripts/eval_profile.py --fused 1 --passes 3 > gpurun_out/r03m_pmc.log 2>&1
