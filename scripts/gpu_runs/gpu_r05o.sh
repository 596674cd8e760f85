#!/bin/bash
# round 5 (o): stream priorities (main chain high / side streams high) and a one-stream executor replay
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/graph_step_probe.py --steps 50 > gpurun_out/r05o_probe.txt 2>&1 || exit $?
GMR_SIDE_PRIO=-1 timeout -k 10 300 python -u scripts/graph_step_probe.py --steps 50 > gpurun_out/r05o_probe_sidehi.txt 2>&1 || exit $?
