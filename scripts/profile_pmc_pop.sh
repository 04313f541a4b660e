#!/bin/bash
# PMC passes (FETCH_SIZE, WRITE_SIZE: one counter per pass, never with trace domains) over the N = 1
# line's population_slerp_7b sub-object (8 x 7B resident, both forms); summary in
# gpurun_out/pmc_pop/pmc_pop_traffic.json.
set -u
cd "$(dirname "$0")/.."
R=$(pwd); OUT=$R/gpurun_out/pmc_pop
mkdir -p $OUT
ARGS="--layout gpt2_small --steps 1 --warmup 0 --cpu-baseline-seconds 0 --bcast-compare 0 --place-candidates 1 --ops population_7b --population-generations 3 --population-reps 10"
# counters on the population passes only (torch's fill launches are not profiled)
KRE="slerp"
for C in FETCH_SIZE WRITE_SIZE; do
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --pmc $C --kernel-include-regex "$KRE" --output-format csv \
      -d $OUT/$C -o pmc -- python3 $R/bench.py --kernel-trace 0 $ARGS > $OUT/$C.log 2>&1); s=$?
  echo "$C pass: status $s"; tail -1 $OUT/$C.log | cut -c1-200
  [ $s -eq 0 ] || exit $s
done
python3 scripts/pmc_population.py $OUT
