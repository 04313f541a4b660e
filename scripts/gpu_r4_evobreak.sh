#!/bin/bash
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r4evobreak; mkdir -p $OUT
timeout -k 10 400 python -u scripts/evomerge_host_breakdown.py --rounds 5 > $OUT/breakdown.json 2> $OUT/breakdown.err || { tail -5 $OUT/breakdown.err; exit 3; }
cat $OUT/breakdown.json
