#!/bin/bash
# Final-format bench, the same command under rocprofv3 (kernel trace + stats), and a marker trace of
# the virtual-rank schedules (roctx ranges). Each GPU step under its own time limit, chained.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out; mkdir -p $OUT
R=$(pwd)
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1 || exit $?
grep '^{' $OUT/bench.log | cut -c1-600
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $R/$OUT/prof_bench -o bench -- python3 $R/bench.py > $R/$OUT/prof_bench.log 2>&1) || exit $?
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --marker-trace --kernel-trace --stats --output-format csv \
    -d $R/$OUT/prof_markers -o vr -- python3 $R/scripts/virtual_schedule_trace.py > $R/$OUT/prof_markers.log 2>&1) || exit $?
grep '^{' $OUT/prof_markers.log
find $OUT/prof_bench $OUT/prof_markers -name "*stats*"
