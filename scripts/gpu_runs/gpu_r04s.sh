#!/bin/bash
# r04s: fused GenRecV1 decoder at 32 / 16 rows per workgroup (tests at both), then the GenRecV1 bench A/B over
# {decoder fused (32 / 16 rows), layer by layer} x {in-batch InfoNCE fused, unfused} and the contrast chunking,
# all without the probe; then a rocprofv3 kernel-stats pass of the default GenRecV1 bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 250 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $T tests/test_decoder_gpu.py > gpurun_out/r04s_tests32.log 2>&1 || { tail -50 gpurun_out/r04s_tests32.log; exit 1; }
tail -2 gpurun_out/r04s_tests32.log
GMR_DEC_ROWS=16 timeout -k 10 300 $T tests/test_decoder_gpu.py > gpurun_out/r04s_tests16.log 2>&1 || { tail -50 gpurun_out/r04s_tests16.log; exit 1; }
tail -2 gpurun_out/r04s_tests16.log
B="python bench.py --model genrecv1 --steps 3 --warmup 1 --no-cpu-baseline --no-probe"
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 $B > gpurun_out/r04s_$tag.json 2> gpurun_out/r04s_$tag.err || { tail -30 gpurun_out/r04s_$tag.err; return 1; }
  echo "$tag $* $(python -c "import json,sys; d=json.load(open('gpurun_out/r04s_$tag.json')); print(d['value'], d['ms_per_step'])")"
}
run d32n1 GMR_DEC_FUSED=1 GMR_NCE_FUSED=1 &&
run d16n1 GMR_DEC_FUSED=1 GMR_DEC_ROWS=16 GMR_NCE_FUSED=1 &&
run d0n1 GMR_DEC_FUSED=0 GMR_NCE_FUSED=1 &&
run d0n0 GMR_DEC_FUSED=0 GMR_NCE_FUSED=0 &&
run d32n0 GMR_DEC_FUSED=1 GMR_NCE_FUSED=0 &&
run d32n1wg GMR_DEC_FUSED=1 GMR_NCE_FUSED=1 GMR_CL_WG_ROWS=128 GMR_CL_WG_TABLE=128 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04s_prof -o run -- python bench.py --model genrecv1 --steps 2 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/r04s_prof.log 2>&1 || { tail -20 gpurun_out/r04s_prof.log; exit 1; }
f=$(find gpurun_out/r04s_prof -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r04s_kernel_stats.csv; cut -d, -f1-5 gpurun_out/r04s_kernel_stats.csv | cut -c1-160 | sed -n 1,30p
