#!/bin/bash
# round 6 (l): GenRecV1 draw kernels at four draws per Philox call (dropout, flip_step, keep masks and the fused
# LayerNorm dropout; two for flip_qsample) (the padded top-K staging of the first run was reverted: conflicts stayed)
# the GenRecV1 / decoder / top-K tests, the GenRecV1 leg A/B against the previous
# library (ablibs/libgmr_y3.so), and the LDS bank-conflict pass over the GenRecV1 leg
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_decoder_gpu.py \
  tests/test_genrec_gpu.py tests/test_genrec_tiktok_gpu.py tests/test_kernels_gpu.py -k "decoder or genrec or topk or draw or tiktok or Layer or layer" \
  > gpurun_out/r06l_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r06l_tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/r06l_tests.log | head -20; exit 1; }
for v in r6l y3 r6l y3; do
  echo "=== $v" >> gpurun_out/r06l_ab.txt
  GMR_HIP_LIB=$PWD/ablibs/libgmr_$v.so GMR_PHASE_TIMES=1 timeout -k 10 300 python -u bench.py --model genrecv1 --no-legs --no-cpu-baseline --no-probe --steps 2 --warmup 1 2>gpurun_out/r06l_err.txt | cut -c1-220 >> gpurun_out/r06l_ab.txt || exit $?
  grep phases gpurun_out/r06l_err.txt | tail -2 >> gpurun_out/r06l_ab.txt
done
cat gpurun_out/r06l_ab.txt
GMR_SERIAL=1 timeout -k 10 -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/r06l_lds -o pmc -- python3 bench.py --model genrecv1 --steps 1 --warmup 1 --no-cpu-baseline --no-probe --no-legs --eval-passes 1 > gpurun_out/r06l_lds.log 2>&1 || exit 1
echo all-done
