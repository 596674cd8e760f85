#!/bin/bash
# SpMM/DiffMM GPU tests, the DiffMM bench (phases + per-shape probe), and a kernel trace of the
# concurrent (non-serial) bench for the GPU-busy analysis of scripts/trace_gaps.py.
set -o pipefail
TAG=${1:-r02j}
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_diffmm_gpu.py tests/test_phases_gpu.py tests/test_genrec_gpu.py -v -m gpu -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_tests.log; grep -E "FAILED|ERROR" gpurun_out/${TAG}_tests.log | head -20; fatal $rc tests
GMR_PHASE_TIMES=1 GMR_PROBE_REPORT=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-legs > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err; rc=$?
head -c 300 gpurun_out/${TAG}_bench.json; echo; grep -A8 "spmm:" gpurun_out/${TAG}_bench.err; grep phases gpurun_out/${TAG}_bench.err | tail -1; fatal $rc bench
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_trace -o tr -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-legs --no-probe > gpurun_out/${TAG}_trace.log 2>&1; rc=$?; fatal $rc rocprof
python scripts/trace_gaps.py $(ls gpurun_out/${TAG}_trace/*kernel_trace.csv | head -1) --steps 40 | tee gpurun_out/${TAG}_gaps.txt
echo all-done
