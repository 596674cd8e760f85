#!/bin/bash
# round 3 final build: default bench line (PMC summaries of this build in profiles/)
cd /root/repo
export TMPDIR=/tmp
GMR_PROBE_REPORT=1 timeout -k 10 700 python -u bench.py > gpurun_out/r03w_bench.json 2> gpurun_out/r03w_bench.err
