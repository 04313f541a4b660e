#!/bin/bash
# r5 PMC re-collection on the final library (every stamped entry the bench line reads).
set -o pipefail
cd "$(dirname "$0")/.."
PMC_TAG=_r5b bash scripts/profile_pmc.sh > gpurun_out/pmc_r5b_main.log 2>&1 || { tail -20 gpurun_out/pmc_r5b_main.log; exit 1; }
bash scripts/profile_pmc_ops.sh > gpurun_out/pmc_r5b_ops.log 2>&1 || { tail -20 gpurun_out/pmc_r5b_ops.log; exit 1; }
bash scripts/profile_pmc_pop.sh > gpurun_out/pmc_r5b_pop.log 2>&1 || { tail -20 gpurun_out/pmc_r5b_pop.log; exit 1; }
bash scripts/profile_pmc_lm.sh > gpurun_out/pmc_r5b_lm.log 2>&1 || { tail -20 gpurun_out/pmc_r5b_lm.log; exit 1; }
echo "pmc done"
