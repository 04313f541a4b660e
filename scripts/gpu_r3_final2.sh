#!/bin/bash
# Round 3 final tree, in the order that lets the bench line carry counters of THIS build: the PMC
# passes first (stamped with the library's sha256), merged into profiles/pmc_traffic.json (a copy
# comes back under gpurun_out/), then bench.py, the same under rocprofv3 --kernel-trace --stats,
# then the whole GPU suite, the SLERP probe and smoke().
set -u
cd "$(dirname "$0")/.."
R=$(pwd); TAG=${TAG:-r3final2}; OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
PMC_TAG=_$TAG ./scripts/profile_pmc.sh > $OUT/pmc.log 2>&1 || { tail -5 $OUT/pmc.log; exit 5; }
./scripts/profile_pmc_ops.sh > $OUT/pmc_ops.log 2>&1 || { tail -5 $OUT/pmc_ops.log; exit 6; }
./scripts/profile_pmc_pop.sh > $OUT/pmc_pop.log 2>&1 || { tail -5 $OUT/pmc_pop.log; exit 6; }
python3 scripts/merge_pmc.py gpurun_out/pmc_$TAG/pmc_traffic.json gpurun_out/pmc_ops/pmc_ops_traffic.json \
    gpurun_out/pmc_pop/pmc_pop_traffic.json || exit 7
cp profiles/pmc_traffic.json $OUT/pmc_traffic.json
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 3; }
tail -c 400 $OUT/bench.json; echo
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $OUT/bkt -o bench -- python3 $R/bench.py --cpu-baseline-seconds 2 > $OUT/bench_under_rocprof.json 2> $OUT/bkt.err) || exit 4
timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1; s=$?
tail -3 $OUT/pytest_gpu.log; [ $s -eq 0 ] || exit $s
# the SLERP forms side by side on the 7B body (arena / tensor-list, speculative / two-pass)
timeout -k 10 300 python scripts/slerp_spec_probe.py --rounds 5 > $OUT/probe_lineage.json 2> $OUT/probe.err || exit 8
timeout -k 10 300 python scripts/slerp_spec_probe.py --rounds 5 --far > $OUT/probe_far.json 2>> $OUT/probe.err || exit 8
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 9
cat $OUT/smoke.log
