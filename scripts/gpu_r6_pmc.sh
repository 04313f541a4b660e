#!/bin/bash
# r6 PMC re-collection on the source-determined library: every stamped entry the bench line reads
# (the 1.3B and 125M fused steps, the ops sub-objects incl. list_form, the 8 x 7B population, the
# EDT-LM generation), FETCH_SIZE and WRITE_SIZE in separate passes, merged into a fresh
# gpurun_out/$TAG/pmc_traffic.json (copied to profiles/pmc_traffic.json after the call).
set -u
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${TAG:-r6pmc}; OUT=gpurun_out/$TAG
mkdir -p $OUT
PMC_TAG=_${TAG}_1p3b bash scripts/profile_pmc.sh > $OUT/pmc_1p3b.log 2>&1 || { tail -5 $OUT/pmc_1p3b.log; exit 5; }
tail -2 $OUT/pmc_1p3b.log
PMC_TAG=_${TAG}_125m BENCH_ARGS="--layout gpt2_small" bash scripts/profile_pmc.sh > $OUT/pmc_125m.log 2>&1 || { tail -5 $OUT/pmc_125m.log; exit 5; }
tail -2 $OUT/pmc_125m.log
bash scripts/profile_pmc_ops.sh > $OUT/pmc_ops.log 2>&1 || { tail -5 $OUT/pmc_ops.log; exit 6; }
bash scripts/profile_pmc_pop.sh > $OUT/pmc_pop.log 2>&1 || { tail -5 $OUT/pmc_pop.log; exit 6; }
bash scripts/profile_pmc_lm.sh > $OUT/pmc_lm.log 2>&1 || { tail -5 $OUT/pmc_lm.log; exit 6; }
python3 scripts/merge_pmc.py --out $OUT/pmc_traffic.json gpurun_out/pmc_${TAG}_1p3b/pmc_traffic.json \
    gpurun_out/pmc_${TAG}_125m/pmc_traffic.json gpurun_out/pmc_ops/pmc_ops_traffic.json \
    gpurun_out/pmc_pop/pmc_pop_traffic.json gpurun_out/pmc_lm/pmc_ops_traffic.json || exit 7
echo done
