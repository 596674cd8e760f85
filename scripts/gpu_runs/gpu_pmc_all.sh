#!/bin/bash
# PMC memory-side traffic for the three bench workloads (DiffMM baby, DiffMM sports, GenRecV1 TikTok).
set -o pipefail
T=${1:-r01h}
bash scripts/pmc_traffic.sh ${T} || exit 1
bash scripts/pmc_traffic.sh ${T}_sports --shape sports || exit 1
bash scripts/pmc_traffic.sh ${T}_genrec --model genrecv1 || exit 1
echo all-done
