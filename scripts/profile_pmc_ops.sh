#!/bin/bash
# PMC passes (FETCH_SIZE, WRITE_SIZE: one counter per pass, never with trace domains) over the bench
# line's pair_merge and slerp_7b kernels; summary in gpurun_out/pmc_ops/pmc_ops_traffic.json.
set -u
cd "$(dirname "$0")/.."
R=$(pwd); OUT=$R/gpurun_out/pmc_ops
mkdir -p $OUT
ARGS="--steps 3 --warmup 1 --cpu-baseline-seconds 0 --ops-cpu-seconds 0 --bcast-compare 0 --place-candidates 1 --ops list_form,configs1_125m,pair_merge,slerp_7b --list-same-memory 0"
# counters on the measured kernels only (torch's fill / cast launches are not profiled)
KRE="outer|pair_kernel|pair_sums|slerp"
for C in FETCH_SIZE WRITE_SIZE; do
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --pmc $C --kernel-include-regex "$KRE" --output-format csv \
      -d $OUT/$C -o pmc -- python3 $R/bench.py --kernel-trace 0 $ARGS > $OUT/$C.log 2>&1); s=$?
  echo "$C pass: status $s"; tail -1 $OUT/$C.log | cut -c1-200
  [ $s -eq 0 ] || exit $s
done
python3 scripts/pmc_ops.py $OUT
