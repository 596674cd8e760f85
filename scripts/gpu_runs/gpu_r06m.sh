#!/bin/bash
# round 6 (m): the GenRecV1 draw kernels at four draws per Philox call (dropout, flip_step; two for
# flip_qsample): decoder / GenRecV1 tests on this library, then per-kernel durations (rocprofv3 --stats, serial
# streams) of the GenRecV1 leg on this library (r6l) and on the previous one (y3)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_decoder_gpu.py \
  tests/test_genrec_gpu.py tests/test_genrec_tiktok_gpu.py tests/test_dist_gpu.py > gpurun_out/r06m_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r06m_tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/r06m_tests.log | head -20; exit 1; }
for v in r6l y3; do
  GMR_HIP_LIB=$PWD/ablibs/libgmr_$v.so GMR_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06m_$v -o prof -- python3 bench.py --model genrecv1 --no-legs --no-cpu-baseline --no-probe --steps 2 --warmup 1 > gpurun_out/r06m_$v.log 2>&1 || exit 1
done
for v in r6l y3; do
  echo "== $v"; grep -E "dropout_kernel|flip_step_kernel|flip_qsample_kernel|ln_fwd_kernel|xattn_fwd" gpurun_out/r06m_$v/*kernel_stats.csv | cut -d, -f1-6
done
echo all-done
