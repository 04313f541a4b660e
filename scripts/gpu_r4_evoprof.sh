#!/bin/bash
# r4: where the EVOMERGE surface's host time goes (cProfile of one merge at 7B, after the timed rounds)
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r4evoprof; mkdir -p $OUT
timeout -k 10 400 python -u scripts/evomerge_probe.py --rounds 3 --profile > $OUT/evomerge.json 2> $OUT/evomerge.err || { tail -5 $OUT/evomerge.err; exit 3; }
cat $OUT/evomerge.json; grep -v amdgpu $OUT/evomerge.err | head -40
