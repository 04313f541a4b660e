#!/bin/bash
# r5 PMC re-collection on the final library: the main step, the ops sub-objects (list_form
# included), the roulette population, and the needed-sums counters on two drawn generations.
set -o pipefail
cd "$(dirname "$0")/.."
if [ "${SKIP_MAIN:-0}" != 1 ]; then
  PMC_TAG=_r5 bash scripts/profile_pmc.sh > gpurun_out/pmc_r5_main.log 2>&1 || { tail -20 gpurun_out/pmc_r5_main.log; exit 1; }
  tail -3 gpurun_out/pmc_r5_main.log
fi
bash scripts/profile_pmc_ops.sh > gpurun_out/pmc_r5_ops.log 2>&1 || { tail -20 gpurun_out/pmc_r5_ops.log; exit 1; }
tail -3 gpurun_out/pmc_r5_ops.log
bash scripts/profile_pmc_pop.sh > gpurun_out/pmc_r5_pop.log 2>&1 || { tail -20 gpurun_out/pmc_r5_pop.log; exit 1; }
tail -3 gpurun_out/pmc_r5_pop.log
TAG=r5pmc GRAPH=0 bash scripts/pmc_need_counters.sh > gpurun_out/pmc_r5_need0.log 2>&1 || { tail -20 gpurun_out/pmc_r5_need0.log; exit 1; }
TAG=r5pmc GRAPH=2 bash scripts/pmc_need_counters.sh > gpurun_out/pmc_r5_need2.log 2>&1 || { tail -20 gpurun_out/pmc_r5_need2.log; exit 1; }
tail -3 gpurun_out/pmc_r5_need0.log gpurun_out/pmc_r5_need2.log
