#!/bin/bash
# HBM traffic of the fused outer-step kernel from PMC counters, one counter group per pass
# (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE cannot share a pass; never with trace domains).
set -u
cd "$(dirname "$0")/.."
R=$(pwd); OUT=$R/gpurun_out/pmc${PMC_TAG:-}
mkdir -p $OUT
# only the DiLoCo step's launches: no sub-object workloads (the 125M step and the fused broadcast
# share the outer_kernel name the summary filters on)
ARGS="--steps 3 --warmup 1 --cpu-baseline-seconds 0 --ops none --bcast-compare 0 ${BENCH_ARGS:-}"
for C in FETCH_SIZE WRITE_SIZE; do
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --pmc $C --output-format csv \
      -d $OUT/$C -o pmc -- python3 $R/bench.py --kernel-trace 0 $ARGS > $OUT/$C.log 2>&1); s=$?
  echo "$C pass: status $s"; tail -2 $OUT/$C.log
  [ $s -eq 0 ] || exit $s
done
python3 scripts/pmc_summary.py $OUT ${BENCH_ARGS:-}
