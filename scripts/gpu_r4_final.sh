#!/bin/bash
# Round 4 final tree, part A, in the order that lets the bench line carry counters of THIS build:
# the PMC passes first (stamped with the library's sha256), merged into profiles/pmc_traffic.json
# (a copy comes back under gpurun_out/), then bench.py and the same under rocprofv3
# --kernel-trace --stats. Part B (gpu_r4_final_b.sh): GPU suite, probes, smoke.
set -u
cd "$(dirname "$0")/.."
R=$(pwd); TAG=${TAG:-r4final}; OUT=$R/gpurun_out/$TAG
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
echo done
