#!/bin/bash
# Round 3: the wave-slot SLERP sums. GPU suite, then the 7B probe in three fresh processes
# (allocation draws) and under rocprofv3 --kernel-trace --stats.
set -u
cd "$(dirname "$0")/.."
R=$(pwd); OUT=$R/gpurun_out/${TAG:-r3b}
mkdir -p $OUT
if [ "${SUITE:-1}" = "1" ]; then
  echo "== pytest -m gpu"
  EDT_RECORD_DIR=$OUT timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread \
      ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1; s=$?
  tail -15 $OUT/pytest_gpu.log; [ $s -le 1 ] || exit $s
fi
for i in 1 2 3; do
  timeout -k 10 300 python scripts/slerp_spec_probe.py ${PROBE_ARGS:-} >> $OUT/probe.jsonl 2>> $OUT/probe.err || exit 3
done
cat $OUT/probe.jsonl
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $OUT/kt -o probe -- python3 $R/scripts/slerp_spec_probe.py --rounds 3 ${PROBE_ARGS:-} > $OUT/kt.log 2>&1); s=$?
tail -1 $OUT/kt.log; grep -E "pair_sums|lerp_kernel|blend_kernel|slot_reduce|coef" $OUT/kt/probe_kernel_stats.csv | cut -d, -f1-4
echo "== done $s"
