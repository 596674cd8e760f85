#!/bin/bash
# r04l: fused eval with the early-exit compaction + scalar-skip filter, fp32 and split-bf16 scores:
# kernel tests, the by-position reference tests (baby, TikTok GenRecV1), microbenchmark both forms.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 250 --timeout-method thread -p no:cacheprovider \
  tests/test_score_topk_gpu.py tests/test_baby_gpu.py tests/test_genrec_tiktok_gpu.py > gpurun_out/r04l_tests.log 2>&1 || { tail -40 gpurun_out/r04l_tests.log; exit 1; }
tail -3 gpurun_out/r04l_tests.log
GMR_EVAL_X6=0 timeout -k 10 120 python scripts/score_topk_bench.py > gpurun_out/r04l_topk.txt 2>&1 || { cat gpurun_out/r04l_topk.txt; exit 1; }
GMR_EVAL_X6=1 timeout -k 10 120 python scripts/score_topk_bench.py >> gpurun_out/r04l_topk.txt 2>&1 || { cat gpurun_out/r04l_topk.txt; exit 1; }
cat gpurun_out/r04l_topk.txt
timeout -k 10 -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d gpurun_out/r04l_pmc1 -o pmc -- python3 scripts/score_topk_bench.py --reps 3 > gpurun_out/r04l_pmc1.log 2>&1 || { tail -20 gpurun_out/r04l_pmc1.log; exit 1; }
python3 scripts/pmcsum.py gpurun_out/r04l_pmc1/pmc_counter_collection.csv --filter score_topk > gpurun_out/r04l_pmc.txt 2>&1; cat gpurun_out/r04l_pmc.txt
