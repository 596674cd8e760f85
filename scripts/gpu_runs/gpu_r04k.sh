#!/bin/bash
# r04k: DiffRec baby-shape training fixture test; sports-shape phase times (DESIGN section 6
# projection); fused-eval microbenchmark + SQ counters.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread -p no:cacheprovider \
  tests/test_diffrec_baby_gpu.py tests/test_baby_gpu.py -k "diffrec or p_sample" > gpurun_out/r04k_tests.log 2>&1 || { tail -40 gpurun_out/r04k_tests.log; exit 1; }
tail -3 gpurun_out/r04k_tests.log
timeout -k 10 120 python scripts/score_topk_bench.py > gpurun_out/r04k_topk.txt 2>&1 || { cat gpurun_out/r04k_topk.txt; exit 1; }
cat gpurun_out/r04k_topk.txt
timeout -k 10 150 python scripts/blas_calib.py > gpurun_out/r04k_blas.txt 2>&1 || { cat gpurun_out/r04k_blas.txt; exit 1; }
cat gpurun_out/r04k_blas.txt
timeout -k 10 -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d gpurun_out/r04k_pmc1 -o pmc -- python3 scripts/score_topk_bench.py --reps 3 > gpurun_out/r04k_pmc1.log 2>&1 || { tail -20 gpurun_out/r04k_pmc1.log; exit 1; }
timeout -k 10 -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_WAVES --output-format csv -d gpurun_out/r04k_pmc2 -o pmc -- python3 scripts/score_topk_bench.py --reps 3 > gpurun_out/r04k_pmc2.log 2>&1 || { tail -20 gpurun_out/r04k_pmc2.log; exit 1; }
python3 scripts/pmcsum.py gpurun_out/r04k_pmc1/pmc_counter_collection.csv gpurun_out/r04k_pmc2/pmc_counter_collection.csv > gpurun_out/r04k_pmc.txt 2>&1; cat gpurun_out/r04k_pmc.txt | head -40
GMR_PHASE_TIMES=1 timeout -k 10 300 python bench.py --shape sports --steps 2 --warmup 1 --no-legs --no-cpu-baseline --no-probe > gpurun_out/r04k_sports.json 2> gpurun_out/r04k_sports.err || { tail -20 gpurun_out/r04k_sports.err; exit 1; }
grep phases gpurun_out/r04k_sports.err | tail -4; cut -c1-400 gpurun_out/r04k_sports.json
