#!/bin/bash
# Round 3: the on-chip-hold SLERP form (edt_slerp_merge_hold) — parity tests, then the 7B far /
# lineage probe (hold timed beside the two-pass form, checked bit for bit), then a kernel trace.
set -u
cd "$(dirname "$0")/.."
R=$(pwd); OUT=$R/gpurun_out/${TAG:-r3hold}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -m gpu --timeout 120 --timeout-method thread \
    -k "hold or slerp" > $OUT/pytest_hold.log 2>&1; s=$?
tail -4 $OUT/pytest_hold.log; [ $s -eq 0 ] || exit $s
timeout -k 10 300 python scripts/slerp_spec_probe.py --rounds 5 --far > $OUT/probe_far.json 2> $OUT/probe.err || exit 3
cat $OUT/probe_far.json
timeout -k 10 300 python scripts/slerp_spec_probe.py --rounds 5 > $OUT/probe_lineage.json 2>> $OUT/probe.err || exit 3
cat $OUT/probe_lineage.json
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $OUT/kt -o probe -- python3 $R/scripts/slerp_spec_probe.py --rounds 3 --far > $OUT/kt.log 2>&1) || exit 4
grep -E "hold|pair_sums|blend|tree_reduce|coef" $OUT/kt/probe_kernel_stats.csv | cut -d, -f1-4
