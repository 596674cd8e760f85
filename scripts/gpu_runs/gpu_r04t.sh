#!/bin/bash
# r04t: xattn backward (parallel dbv' reduction), contrast fixup with batched chunk loads, GenRecV1 suites;
# GenRecV1 bench (layer-by-layer decoder default) with the probe report; its kernel stats; DiffMM headline.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 250 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_decoder_gpu.py tests/test_genrec_gpu.py tests/test_genrec_tiktok_gpu.py tests/test_kernels_gpu.py -k "decoder or genrec or GenRec or xattn or contrast or denoiser" > gpurun_out/r04t_tests.log 2>&1 || { tail -50 gpurun_out/r04t_tests.log; exit 1; }
tail -2 gpurun_out/r04t_tests.log
GMR_PROBE_REPORT=1 timeout -k 10 300 python bench.py --model genrecv1 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r04t_genrec.json 2> gpurun_out/r04t_genrec.err || { tail -30 gpurun_out/r04t_genrec.err; exit 1; }
cut -c1-260 gpurun_out/r04t_genrec.json; grep -E "^---" gpurun_out/r04t_genrec.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04t_prof -o run -- python bench.py --model genrecv1 --steps 2 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/r04t_prof.log 2>&1 || { tail -20 gpurun_out/r04t_prof.log; exit 1; }
f=$(find gpurun_out/r04t_prof -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r04t_genrec_kernel_stats.csv
GMR_PROBE_REPORT=1 timeout -k 10 300 python bench.py --model diffmm --no-legs --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r04t_diffmm.json 2> gpurun_out/r04t_diffmm.err || { tail -30 gpurun_out/r04t_diffmm.err; exit 1; }
cut -c1-260 gpurun_out/r04t_diffmm.json; grep -E "^---" gpurun_out/r04t_diffmm.err
