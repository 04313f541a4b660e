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
# the N > 1 line's code path at world 1 over RCCL (value, parity of the schedule and of the sharded
# population child; the 8-GPU runs are the driver's)
timeout -k 10 600 python -u bench.py --gpus 1 --sharded --steps 5 --warmup 2 --cpu-baseline-seconds 1 \
    --config-companions 0 > $OUT/bench_sharded_world1.json 2> $OUT/bench_sharded_world1.err || { tail -5 $OUT/bench_sharded_world1.err; exit 12; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('parity', d.get('parity')); print('pop parity', {k: v.get('parity') for k, v in d.get('population_slerp_7b', {}).items() if isinstance(v, dict)})" $OUT/bench_sharded_world1.json
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 11
cat $OUT/smoke.log
echo done
