#!/bin/bash
# r5: PMC passes (FETCH_SIZE, WRITE_SIZE, separate runs) over the N = 1 line's lm_population
# sub-object only (the EDT-LM generation's pair_population_kernel); summary via pmc_ops.py.
set -u
cd "$(dirname "$0")/.."
R=$(pwd); OUT=$R/gpurun_out/pmc_lm
mkdir -p $OUT
ARGS="--layout gpt2_small --steps 1 --warmup 0 --cpu-baseline-seconds 0 --ops-cpu-seconds 0 --bcast-compare 0 --place-candidates 1 --ops lm_population"
KRE="pair_population"
for C in FETCH_SIZE WRITE_SIZE; do
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --pmc $C --kernel-include-regex "$KRE" --output-format csv \
      -d $OUT/$C -o pmc -- python3 $R/bench.py --kernel-trace 0 $ARGS > $OUT/$C.log 2>&1); s=$?
  echo "$C pass: status $s"; tail -1 $OUT/$C.log | cut -c1-200
  [ $s -eq 0 ] || exit $s
done
python3 scripts/pmc_ops.py $OUT
