#!/bin/bash
# round 6 (d): the rec-step fusions and the scheduled InfoNCE passes (GMR_CL_SCHED): full GPU suite, the
# InfoNCE microbenchmark per schedule, the epoch per schedule, and a kernel trace of one epoch
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q -s --timeout 200 --timeout-method thread tests/test_diffmm_train_gpu.py -m gpu \
  -k "diffusion_step" > gpurun_out/r06d_gc.log 2>&1
grep -E "^\[|passed|failed" gpurun_out/r06d_gc.log
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu -k "not diffusion_step" \
  > gpurun_out/r06d_tests.log 2>&1 || { tail -60 gpurun_out/r06d_tests.log; exit 1; }
tail -2 gpurun_out/r06d_tests.log
for s in 0 1 2 0 1 2; do
  echo "=== GMR_CL_SCHED=$s" >> gpurun_out/r06d_cl.txt
  GMR_CL_SCHED=$s timeout -k 10 120 python -u scripts/contrast_bench.py 2>&1 | grep -v amdgpu.ids >> gpurun_out/r06d_cl.txt || exit $?
done
cat gpurun_out/r06d_cl.txt
for s in 0 1 0 1; do
  echo "=== GMR_CL_SCHED=$s" >> gpurun_out/r06d_ab.txt
  GMR_CL_SCHED=$s GMR_PHASE_TIMES=1 timeout -k 10 200 python -u bench.py --model diffmm --no-legs --no-cpu-baseline --no-probe --steps 5 --warmup 1 2>gpurun_out/r06d_err.txt | cut -c1-200 >> gpurun_out/r06d_ab.txt || exit $?
  grep phases gpurun_out/r06d_err.txt | tail -3 >> gpurun_out/r06d_ab.txt
done
cat gpurun_out/r06d_ab.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r06d_trace -o tr -- python3 bench.py --model diffmm --no-legs --no-cpu-baseline --no-probe --steps 1 --warmup 1 --eval-passes 1 > gpurun_out/r06d_trace.log 2>&1 || { tail -20 gpurun_out/r06d_trace.log; exit 1; }
python scripts/trace_gaps.py gpurun_out/r06d_trace/*kernel_trace.csv --steps 20 > gpurun_out/r06d_gaps.txt 2>&1
head -40 gpurun_out/r06d_gaps.txt
echo all-done
