#!/bin/bash
# Round 4 final tree, part B: the whole GPU suite, the SLERP probes (lineage / far), the population
# probe under rocprofv3 --kernel-trace --stats (the Gram pass's time), the EVOMERGE surface probe,
# smoke().
set -u
cd "$(dirname "$0")/.."
R=$(pwd); TAG=${TAG:-r4final}; OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $OUT/pytest_gpu.log 2>&1; s=$?
tail -3 $OUT/pytest_gpu.log; [ $s -eq 0 ] || exit $s
timeout -k 10 300 python -u scripts/slerp_spec_probe.py --rounds 6 > $OUT/probe_lineage.json 2> $OUT/probe.err || exit 8
timeout -k 10 300 python -u scripts/slerp_spec_probe.py --rounds 6 --far > $OUT/probe_far.json 2>> $OUT/probe.err || exit 8
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $OUT/pop -o pop -- python3 $R/scripts/pop_slerp_probe.py --rounds 3 > $OUT/pop_probe.log 2>&1) || exit 9
timeout -k 10 400 python -u scripts/evomerge_probe.py --rounds 5 > $OUT/evomerge_lineage.json 2> $OUT/evomerge.err || exit 10
timeout -k 10 400 python -u scripts/evomerge_probe.py --rounds 5 --far > $OUT/evomerge_far.json 2>> $OUT/evomerge.err || exit 10
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 11
cat $OUT/smoke.log
echo done
