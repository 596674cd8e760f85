#!/bin/bash
# Full GPU test suite + DiffMM bench (default workload) + GenRecV1 bench; logs under gpurun_out/.
set -o pipefail
TAG=${1:-both}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" gpurun_out/${TAG}_tests.log | head -20; tail -5 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_bench_dmm.json 2> gpurun_out/${TAG}_bench_dmm.err || { echo "dmm bench failed"; tail -20 gpurun_out/${TAG}_bench_dmm.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench_dmm.json'));print('diffmm', d['value'], d['ms_per_step'], d['eval_users_per_s'])"
timeout -k 10 400 python bench.py --model genrecv1 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_bench_gr.json 2> gpurun_out/${TAG}_bench_gr.err || { echo "gr bench failed"; tail -20 gpurun_out/${TAG}_bench_gr.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench_gr.json'));print('genrecv1', d['value'], d['ms_per_step'], d['eval_users_per_s'])"
