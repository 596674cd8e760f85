#!/bin/bash
# r04x: LayerNorm with the residual-branch dropout drawn in-kernel (gmr_layernorm_drop_fwd): decoder / GenRecV1
# tests, then the GenRecV1 bench twice.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 250 --timeout-method thread -p no:cacheprovider tests/test_decoder_gpu.py tests/test_genrec_gpu.py tests/test_genrec_tiktok_gpu.py tests/test_tiktok_gpu.py tests/test_dist_gpu.py -k "decoder or layernorm or genrec or GenRec or tiktok or denoiser or dp2" > gpurun_out/r04x_tests.log 2>&1 || { tail -50 gpurun_out/r04x_tests.log; exit 1; }
tail -2 gpurun_out/r04x_tests.log
for r in a b; do
timeout -k 10 300 python bench.py --model genrecv1 --steps 3 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/r04x_genrec_$r.json 2> gpurun_out/r04x_genrec_$r.err || { tail -20 gpurun_out/r04x_genrec_$r.err; exit 1; }
echo "$r $(python -c "import json; d=json.load(open('gpurun_out/r04x_genrec_$r.json')); print(d['value'], d['ms_per_step'])")"
done
