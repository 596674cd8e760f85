#!/bin/bash
# r04v: tests for the new defaults (contrast fixup opt-in, 256-deep 64^2 split-K slabs); InfoNCE grid sweep
# (GMR_CL_WG_ROWS / GMR_CL_WG_TABLE) under GMR_CL_PIPE 1 / 0; DiffMM epoch A/B of GMR_CL_PIPE (alternating).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 250 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_kernels_gpu.py tests/test_genrec_gpu.py tests/test_decoder_gpu.py -k "contrast or gemm or x6 or genrec or GenRec or decoder or denoiser" > gpurun_out/r04v_tests.log 2>&1 || { tail -50 gpurun_out/r04v_tests.log; exit 1; }
tail -2 gpurun_out/r04v_tests.log
for p in 0 1; do for wr in 256 512 1024; do for wt in 384 768 1536; do
  echo "[PIPE=$p WG_ROWS=$wr WG_TABLE=$wt] $(GMR_CL_PIPE=$p GMR_CL_WG_ROWS=$wr GMR_CL_WG_TABLE=$wt timeout -k 10 120 python scripts/contrast_bench.py --reps 30 2>&1 | grep us/call | awk '{print $2, $3}' | tr '\n' ' ')" || exit 1
done; done; done > gpurun_out/r04v_contrast_sweep.txt
cat gpurun_out/r04v_contrast_sweep.txt
B="python bench.py --model diffmm --no-legs --steps 5 --warmup 2 --no-cpu-baseline --no-probe"
for r in a b; do for p in 1 0; do
  GMR_CL_PIPE=$p timeout -k 10 300 $B > gpurun_out/r04v_diffmm_p$p$r.json 2> gpurun_out/r04v_diffmm_p$p$r.err || { tail -20 gpurun_out/r04v_diffmm_p$p$r.err; exit 1; }
  echo "pipe=$p ($r) $(python -c "import json; d=json.load(open('gpurun_out/r04v_diffmm_p$p$r.json')); print(d['value'], d['ms_per_step'])")"
done; done
