#!/bin/bash
# Round 3 final-tree measurement: bench.py (N = 1 default line), the same under rocprofv3
# --kernel-trace --stats, the PMC traffic passes of every kernel in the line (stamped with the
# library's sha256), and the SLERP counter passes (spec pass vs lerp).
set -u
cd "$(dirname "$0")/.."
R=$(pwd); OUT=$R/gpurun_out/${TAG:-r3final}
mkdir -p $OUT
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 3; }
tail -c 600 $OUT/bench.json; echo
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $OUT/bkt -o bench -- python3 $R/bench.py --cpu-baseline-seconds 2 > $OUT/bench_under_rocprof.json 2> $OUT/bkt.err) || exit 4
PMC_TAG=_$TAG ./scripts/profile_pmc.sh > $OUT/pmc.log 2>&1 || { tail -5 $OUT/pmc.log; exit 5; }
./scripts/profile_pmc_ops.sh > $OUT/pmc_ops.log 2>&1 || { tail -5 $OUT/pmc_ops.log; exit 6; }
tail -3 $OUT/pmc_ops.log
TAG=$TAG ./scripts/pmc_slerp_counters.sh > $OUT/counters.log 2>&1 || { tail -5 $OUT/counters.log; exit 7; }
echo done
