#!/bin/bash
set -u
cd /root/repo
OUT=gpurun_out/r4gv; mkdir -p $OUT
timeout -k 10 500 python -u scripts/pop_slerp_probe.py --rounds 3 --variants variants_slerp > $OUT/pop_variants.log 2>&1 || { tail -5 $OUT/pop_variants.log; exit 3; }
grep -v "^{" $OUT/pop_variants.log | grep -v "^[EW]20" | tail -12
