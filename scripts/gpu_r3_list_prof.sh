#!/bin/bash
# Round 3: kernel trace of the SLERP forms on the 7B body (lineage parents), arena and tensor-list
# side by side, to split the list form's extra time into kernel and host parts.
set -u
cd "$(dirname "$0")/.."
R=$(pwd); OUT=$R/gpurun_out/${TAG:-r3listprof}
mkdir -p $OUT
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $OUT/kt -o probe -- python3 $R/scripts/slerp_spec_probe.py --rounds 5 > $OUT/kt.log 2>&1); s=$?
grep '"probe"' $OUT/kt.log; echo "rocprof status $s"
python3 scripts/trace_by_grid.py $OUT/kt/probe_kernel_trace.csv > $OUT/by_grid.txt 2>&1; head -20 $OUT/by_grid.txt
