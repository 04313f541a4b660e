#!/bin/bash
# r4: population pass counters on the final build, the bench's ring of children and the probe's matching
set -u
cd "$(dirname "$0")/.."
TAG=r4popc_ring PAIRS=ring ./scripts/pmc_pop_counters.sh > gpurun_out/popc_ring.log 2>&1 || { tail -5 gpurun_out/popc_ring.log; exit 3; }
TAG=r4popc_probe PAIRS=probe ./scripts/pmc_pop_counters.sh > gpurun_out/popc_probe.log 2>&1 || { tail -5 gpurun_out/popc_probe.log; exit 4; }
echo ok
