#!/bin/bash
# round 6 (p): the InfoNCE loss / dP finalize merged into the table reduce's launch (the table pass derives r from
# the rows pass's partials): InfoNCE / rec-step / stream-order / training tests, a kernel trace of the rec step
# (kernels per step), and the epoch A/B against the previous library (ablibs/libgmr_prev.so)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_kernels_gpu.py \
  tests/test_diffmm_gpu.py tests/test_stream_order_gpu.py tests/test_diffmm_train_gpu.py tests/test_phases_gpu.py \
  tests/test_genrec_gpu.py -k "contrast or rec_step or stream or epochs or train or infonce or phase or genrec or nce or baby or sports" \
  > gpurun_out/r06p_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r06p_tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/r06p_tests.log | head -20; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r06p_trace -o tr -- python3 bench.py --model diffmm --no-legs --no-cpu-baseline --no-probe --steps 1 --warmup 1 --eval-passes 1 > gpurun_out/r06p_trace.log 2>&1 || exit 1
python scripts/trace_gaps.py gpurun_out/r06p_trace/*kernel_trace.csv --steps 20 > gpurun_out/r06p_rec_step_trace.txt 2>&1
head -8 gpurun_out/r06p_rec_step_trace.txt
for v in merged prev merged prev; do
  echo "=== $v" >> gpurun_out/r06p_ab.txt
  GMR_HIP_LIB=$PWD/ablibs/libgmr_$v.so GMR_PHASE_TIMES=1 timeout -k 10 200 python -u bench.py --model diffmm --no-legs --no-cpu-baseline --no-probe --steps 5 --warmup 1 2>gpurun_out/r06p_err.txt | cut -c1-200 >> gpurun_out/r06p_ab.txt || exit $?
  grep phases gpurun_out/r06p_err.txt | tail -3 >> gpurun_out/r06p_ab.txt
done
cat gpurun_out/r06p_ab.txt
echo all-done
