#!/bin/bash
# Round 3: the speculative tensor-list SLERP (edt_slerp_merge_list_speculative) — parity tests,
# then the 7B probe (lineage and far parents) with the list forms beside the arena forms.
set -u
cd "$(dirname "$0")/.."
R=$(pwd); OUT=$R/gpurun_out/${TAG:-r3list}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_surfaces.py -x -q -m gpu --timeout 120 \
    --timeout-method thread -k "slerp or list or crossover or evomerge" > $OUT/pytest_list.log 2>&1; s=$?
tail -4 $OUT/pytest_list.log; [ $s -eq 0 ] || exit $s
timeout -k 10 300 python scripts/slerp_spec_probe.py --rounds 5 > $OUT/probe_lineage.json 2> $OUT/probe.err || exit 3
cat $OUT/probe_lineage.json
timeout -k 10 300 python scripts/slerp_spec_probe.py --rounds 5 --far > $OUT/probe_far.json 2>> $OUT/probe.err || exit 3
cat $OUT/probe_far.json
