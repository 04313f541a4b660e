#!/bin/bash
# Round 3: the default bench line (N = 1) and smoke().
set -u
cd "$(dirname "$0")/.."
R=$(pwd); OUT=$R/gpurun_out/${TAG:-r3bench}
mkdir -p $OUT
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 3; }
tail -c 1500 $OUT/bench.json; echo
