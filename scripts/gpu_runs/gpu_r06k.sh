#!/bin/bash
# round 6 (k): full GPU suite + smoke on the current library, the CLN-rows-on-the-InfoNCE-streams A/B
# (GMR_CL_ROWS_SIDE), and host issue vs GPU time per rec step (eager / tape)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_runs/gpu_r06ev_tests.sh r06k || exit 1
for v in 1 0 1 0; do
  echo "=== GMR_CL_ROWS_SIDE=$v" >> gpurun_out/r06k_ab.txt
  GMR_CL_ROWS_SIDE=$v GMR_PHASE_TIMES=1 timeout -k 10 200 python -u bench.py --model diffmm --no-legs --no-cpu-baseline --no-probe --steps 5 --warmup 1 2>gpurun_out/r06k_err.txt | cut -c1-200 >> gpurun_out/r06k_ab.txt || exit $?
  grep phases gpurun_out/r06k_err.txt | tail -3 >> gpurun_out/r06k_ab.txt
done
cat gpurun_out/r06k_ab.txt
for t in "" "--tape"; do
  timeout -k 10 200 python -u scripts/host_vs_gpu_probe.py --steps 8 $t >> gpurun_out/r06k_host_vs_gpu.log 2>&1 || exit $?
done
grep rep gpurun_out/r06k_host_vs_gpu.log
echo all-done
