#!/bin/bash
# r5 PMC re-collection on the final library (every stamped entry the bench line reads).
set -o pipefail
cd "$(dirname "$0")/.."
PMC_TAG=${PMC_TAG:-_r5b} bash scripts/profile_pmc.sh > gpurun_out/pmc${PMC_TAG:-_r5b}_main.log 2>&1 || { tail -20 gpurun_out/pmc${PMC_TAG:-_r5b}_main.log; exit 1; }
bash scripts/profile_pmc_ops.sh > gpurun_out/pmc${PMC_TAG:-_r5b}_ops.log 2>&1 || { tail -20 gpurun_out/pmc${PMC_TAG:-_r5b}_ops.log; exit 1; }
bash scripts/profile_pmc_pop.sh > gpurun_out/pmc${PMC_TAG:-_r5b}_pop.log 2>&1 || { tail -20 gpurun_out/pmc${PMC_TAG:-_r5b}_pop.log; exit 1; }
bash scripts/profile_pmc_lm.sh > gpurun_out/pmc${PMC_TAG:-_r5b}_lm.log 2>&1 || { tail -20 gpurun_out/pmc${PMC_TAG:-_r5b}_lm.log; exit 1; }
echo "pmc done"
