#!/bin/bash
# Round 4 measurement batch: GPU suite, SLERP probes (lineage + far), the EVOMERGE surface at 7B,
# and the default bench line. Each step under its own time limit; the first failure ends the call.
set -u
cd "$(dirname "$0")/.."
R=$(pwd); OUT=$R/gpurun_out/${TAG:-r4batch}
mkdir -p $OUT
if [ "${SUITE:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=10 -q --timeout 300 --timeout-method thread \
      -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1; s=$?
  tail -4 $OUT/pytest_gpu.log; [ $s -eq 0 ] || exit $s
fi
timeout -k 10 300 python -u scripts/slerp_spec_probe.py --rounds 6 > $OUT/probe_lineage.json 2> $OUT/probe_lineage.err || { tail -5 $OUT/probe_lineage.err; exit 3; }
timeout -k 10 300 python -u scripts/slerp_spec_probe.py --rounds 6 --far > $OUT/probe_far.json 2> $OUT/probe_far.err || { tail -5 $OUT/probe_far.err; exit 4; }
timeout -k 10 600 python -u scripts/evomerge_probe.py --rounds 5 > $OUT/evomerge_lineage.json 2> $OUT/evomerge_lineage.err || { tail -5 $OUT/evomerge_lineage.err; exit 5; }
timeout -k 10 600 python -u scripts/evomerge_probe.py --rounds 5 --far > $OUT/evomerge_far.json 2> $OUT/evomerge_far.err || { tail -5 $OUT/evomerge_far.err; exit 6; }
if [ "${POP:-1}" = 1 ]; then
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
      -d $OUT/pop -o pop -- python3 $R/scripts/pop_slerp_probe.py --rounds 3 > $OUT/pop_probe.log 2>&1) || { tail -5 $OUT/pop_probe.log; exit 8; }
  grep -v "^[EW]20" $OUT/pop_probe.log | tail -3
fi
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 7; }
  tail -c 400 $OUT/bench.json; echo
fi
echo done
