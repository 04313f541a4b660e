#!/bin/bash
# Round 3: the whole GPU suite, then the 7B SLERP probe in two fresh processes and under rocprofv3.
set -u
cd "$(dirname "$0")/.."
R=$(pwd); OUT=$R/gpurun_out/${TAG:-r3g}
mkdir -p $OUT
EDT_RECORD_DIR=$OUT timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread \
    ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1; s=$?
tail -6 $OUT/pytest_gpu.log; [ $s -le 1 ] || exit $s
for far in "" "--far"; do
  V=""; [ -d variants_slerp ] && V="--variants variants_slerp"      # build-time variants, if built
  timeout -k 10 300 python scripts/slerp_spec_probe.py --rounds 5 $far $V >> $OUT/probe.jsonl 2>> $OUT/probe.err || exit 3
done
cat $OUT/probe.jsonl
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $OUT/kt -o probe -- python3 $R/scripts/slerp_spec_probe.py --rounds 3 > $OUT/kt.log 2>&1) || exit 4
grep -E "pair_sums|lerp_kernel|blend_kernel|tree_reduce|coef" $OUT/kt/probe_kernel_stats.csv | cut -d, -f1-4
exit $s
