#!/bin/bash
# round-6 evidence, part 3: the default bench line (with the legs and cpu_baseline; reads part 2's PMC
# summaries), a kernel trace of the rec step, host issue vs GPU time per step, and rank 0's measured work at
# W = 1, 2, 4, 8
# usage: bash scripts/gpu_runs/gpu_r06ev_bench.sh <tag>
set -o pipefail
TAG=${1:-r06ev}
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { case $1 in 0) ;; *) echo "fatal exit $1 in $2"; tail -20 gpurun_out/${TAG}_$2.log 2>/dev/null; exit 1;; esac; }
sha256sum generative-multimodal-recommendation_amd/gmr/libgmr_hip.so | tee gpurun_out/${TAG}_lib_sha.txt
GMR_PROBE_REPORT=1 timeout -k 10 700 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.log; fatal $? bench
cut -c1-400 gpurun_out/${TAG}_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_trace -o tr -- python3 bench.py --model diffmm --no-legs --no-cpu-baseline --no-probe --steps 1 --warmup 1 --eval-passes 1 > gpurun_out/${TAG}_trace.log 2>&1; fatal $? trace
python scripts/trace_gaps.py gpurun_out/${TAG}_trace/*kernel_trace.csv --steps 20 > gpurun_out/${TAG}_rec_step_trace.txt 2>&1
head -30 gpurun_out/${TAG}_rec_step_trace.txt
for t in "" "--tape"; do
  timeout -k 10 200 python -u scripts/host_vs_gpu_probe.py --steps 8 $t >> gpurun_out/${TAG}_host_vs_gpu.log 2>&1; fatal $? host_vs_gpu
done
grep rep gpurun_out/${TAG}_host_vs_gpu.log
timeout -k 10 400 python -u scripts/dp_shard_probe.py --worlds 1,2,4,8 --epochs 3 > gpurun_out/${TAG}_dp_shard.log 2>&1; fatal $? dp_shard
tail -12 gpurun_out/${TAG}_dp_shard.log
echo all-done
