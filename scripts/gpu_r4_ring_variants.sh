#!/bin/bash
# r4: build-time variants of the ring passes on the bench's ring of children (bits checked)
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r4rv; mkdir -p $OUT
timeout -k 10 500 python -u scripts/pop_slerp_probe.py --rounds 3 --pairs ring --variants variants_slerp > $OUT/pop_variants.log 2>&1 || { tail -5 $OUT/pop_variants.log; exit 3; }
grep -v "^{" $OUT/pop_variants.log | grep -v "^[EW]20" | grep -v amdgpu | tail -12
