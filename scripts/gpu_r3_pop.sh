#!/bin/bash
# The resident 8 x 7B SLERP population (BASELINE configs[4]) timed warm in every form, then the
# same probe under rocprofv3 --kernel-trace --stats for the per-kernel split.
set -u
cd "$(dirname "$0")/.."
R=$(pwd); OUT=$R/gpurun_out/${TAG:-r3p}
mkdir -p $OUT
V=""; [ -d variants_slerp ] && V="--variants variants_slerp"
timeout -k 10 600 python -u scripts/pop_slerp_probe.py --rounds 3 $V > $OUT/pop_probe.log 2>&1 || { tail -20 $OUT/pop_probe.log; exit 3; }
tail -1 $OUT/pop_probe.log
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $OUT/pkt -o pop -- python3 $R/scripts/pop_slerp_probe.py --rounds 1 > $OUT/pkt.log 2>&1) || exit 4
grep -E "slerp|pair_sums|tree_reduce|gram" $OUT/pkt/pop_kernel_stats.csv | cut -d, -f1-4 | cut -c1-150
