#!/bin/bash
# HBM bytes per launch of the population SLERP kernels at 8 x 7B (pop_slerp_probe.py --rounds 1,
# every form): FETCH_SIZE and WRITE_SIZE in separate passes, never with trace domains.
set -u
cd "$(dirname "$0")/.."
R=$(pwd); OUT=$R/gpurun_out/${TAG:-r3pp}/pmc
mkdir -p $OUT
for C in FETCH_SIZE WRITE_SIZE; do
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --pmc $C --output-format csv \
      -d $OUT/$C -o pmc -- python3 $R/scripts/pop_slerp_probe.py --rounds 1 > $OUT/$C.log 2>&1); s=$?
  echo "$C pass: status $s"; [ $s -eq 0 ] || exit $s
done
python3 scripts/pmc_by_kernel.py $OUT > $OUT/by_kernel.json; grep -A3 "pop_stats\|gram_kernel\|blend_mm\|blend_population" $OUT/by_kernel.json | head -40
