#!/bin/bash
# r4: population pass counters on the final build, the bench's ring of children and the probe's
# matching; only the summaries are kept (the per-dispatch CSVs exceed gpurun's copy-back limit)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r4popc2
for P in ring probe; do
  TAG=r4popc_$P PAIRS=$P ./scripts/pmc_pop_counters.sh > gpurun_out/r4popc2/$P.log 2>&1; s=$?
  cp gpurun_out/r4popc_$P/counters/summary.json gpurun_out/r4popc2/summary_$P.json 2>/dev/null
  rm -rf gpurun_out/r4popc_$P
  [ $s -eq 0 ] || { tail -5 gpurun_out/r4popc2/$P.log; exit 3; }
done
echo ok
