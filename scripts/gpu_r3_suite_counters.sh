#!/bin/bash
# The GPU suite + 7B SLERP probe (gpu_r3_suite.sh), then the SLERP counter passes (pmc_slerp_counters.sh).
set -u
cd "$(dirname "$0")/.."
./scripts/gpu_r3_suite.sh && ./scripts/pmc_slerp_counters.sh
