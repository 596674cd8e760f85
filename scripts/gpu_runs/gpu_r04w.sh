#!/bin/bash
# r04w: the whole -m gpu suite on the current library (k-means++ pick / greedy wave sums, SpMM hub fences,
# contrast fixup opt-in, 64^2 slabs), then the GenRecV1 bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 250 --timeout-method thread -p no:cacheprovider > gpurun_out/r04w_tests.log 2>&1 || { tail -60 gpurun_out/r04w_tests.log; exit 1; }
tail -2 gpurun_out/r04w_tests.log
timeout -k 10 300 python bench.py --model genrecv1 --steps 3 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/r04w_genrec.json 2> gpurun_out/r04w_genrec.err || { tail -20 gpurun_out/r04w_genrec.err; exit 1; }
cut -c1-250 gpurun_out/r04w_genrec.json
