#!/bin/bash
# PMC memory-side traffic for GenRecV1 TikTok and DiffMM sports (bench without HIP-event probes).
set -o pipefail
T=${1:-r01i}
bash scripts/pmc_traffic.sh ${T}_genrec --model genrecv1 || exit 1
bash scripts/pmc_traffic.sh ${T}_sports --shape sports || exit 1
echo all-done
