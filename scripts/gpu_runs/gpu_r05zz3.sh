#!/bin/bash
# round 5 (zz3): both InfoNCE convert halves conflict-free (row-major rotation added): the zz checks again
# contrast microbenchmark and the epoch, alternating with the r05ev6 library (ablibs/libgmr_r05ev6.so)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py \
  tests/test_diffmm_gpu.py tests/test_diffmm_baby_train_gpu.py -k "contrast or cl or diffmm" -m gpu > gpurun_out/r05zz3_tests.log 2>&1 || exit $?
for lib in ev6 new ev6 new; do
  if [ $lib = ev6 ]; then L=ablibs/libgmr_r05ev6.so; else L=generative-multimodal-recommendation_amd/gmr/libgmr_hip.so; fi
  echo "=== $lib" >> gpurun_out/r05zz3_bench.txt
  GMR_HIP_LIB=$L timeout -k 10 200 python -u scripts/contrast_bench.py 2>&1 | grep -v amdgpu.ids >> gpurun_out/r05zz3_bench.txt || exit $?
done
for lib in ev6 new ev6 new ev6 new; do
  if [ $lib = ev6 ]; then L=ablibs/libgmr_r05ev6.so; else L=generative-multimodal-recommendation_amd/gmr/libgmr_hip.so; fi
  echo "=== $lib" >> gpurun_out/r05zz3_ab.txt
  GMR_HIP_LIB=$L GMR_PHASE_TIMES=1 timeout -k 10 200 python -u bench.py --model diffmm --no-legs --no-cpu-baseline --no-probe --steps 5 --warmup 1 2>gpurun_out/r05zz3_err.txt | cut -c1-200 >> gpurun_out/r05zz3_ab.txt || exit $?
  grep phases gpurun_out/r05zz3_err.txt | tail -2 >> gpurun_out/r05zz3_ab.txt
done
timeout -k 10 -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/r05zz3_lds -o pmc -- python3 bench.py --model diffmm --steps 1 --warmup 1 --no-cpu-baseline --no-probe --no-legs --eval-passes 1 > gpurun_out/r05zz3_lds.log 2>&1 || exit 1
