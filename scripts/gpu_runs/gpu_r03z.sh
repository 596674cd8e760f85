#!/bin/bash
# round 3: single-launch column sums (GenRecV1 bias gradients): tests + GenRecV1 bench
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_genrec_gpu.py tests/test_diffmm_gpu.py -k "colsum or genrec or denoiser or transformer or diffusion or trainer" > gpurun_out/r03z_tests.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --model genrecv1 --scoring-dtype fp16 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03z_genrec.json 2> gpurun_out/r03z_genrec.err
