#!/bin/bash
# Round 3: the on-chip-hold SLERP form (edt_slerp_merge_hold) — parity tests, then the 7B far
# probe (hold timed beside the two-pass form, checked bit for bit; build-time variants from
# variants_hold/ when present).
set -u
cd "$(dirname "$0")/.."
R=$(pwd); OUT=$R/gpurun_out/${TAG:-r3hold}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -m gpu --timeout 120 --timeout-method thread \
    -k "hold or slerp" > $OUT/pytest_hold.log 2>&1; s=$?
tail -4 $OUT/pytest_hold.log; [ $s -eq 0 ] || exit $s
V=""; [ -d variants_hold ] && V="--variants variants_hold"
timeout -k 10 400 python scripts/slerp_spec_probe.py --rounds 5 --far $V > $OUT/probe_far.json 2> $OUT/probe.err || exit 3
cat $OUT/probe_far.json
