#!/bin/bash
# r6: PMC passes on this library (stamped), the stamped summary installed as profiles/pmc_traffic.json
# on the box (the local copy is made after the call), then the final-tree script.
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${TAG:-r6pmc2}
TAG=$TAG bash scripts/gpu_r6_pmc.sh || exit 1
cp gpurun_out/$TAG/pmc_traffic.json profiles/pmc_traffic.json || exit 1
R6_OUT=${R6_OUT:-r6final2} bash scripts/gpu_r6_final.sh
