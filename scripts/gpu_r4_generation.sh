#!/bin/bash
# r4: one resident generation (population.py, selection -> merges -> swap) at 1.3B x 8 on the final build
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r4gen; mkdir -p $OUT
timeout -k 10 500 python -u scripts/bench_generation.py --layout gpt_1p3b --population 8 --iters 5 \
    --json $OUT/generation_1p3b.json > $OUT/gen.log 2>&1 || { tail -5 $OUT/gen.log; exit 3; }
cat $OUT/generation_1p3b.json | head -c 3000
