#!/bin/bash
# r5: the fused step with non-temporal theta / momentum loads and stores (EDT_NT_RMW=1
# EDT_NT_STORES=1, variant nt_rmw_st) against the shipped build on every op family the switch
# reaches (the stores default of every kernel): outer step (three dtype regimes), the list step,
# lerp / pair merge, one SLERP child, both populations. Interleaved in one process per op.
set -o pipefail
O=gpurun_out/ntrmw
mkdir -p $O
V=default,nt_rmw_st
for spec in "outer f32 f32" "outer f32 bf16" "outer bf16 bf16" "list f32 f32" "stream - -" "slerp - -" "pair_pop - -" "slerp_pop - -"; do
  set -- $spec
  args="--op $1 --variants $V --rounds 5"
  [ "$2" != "-" ] && args="$args --tdt $2 --wdt $3"
  echo "== $spec" | tee -a $O/all.log
  timeout -k 10 300 python3 -u scripts/kernel_variants.py $args >> $O/all.log 2>> $O/err.log || { tail -20 $O/err.log; exit 1; }
done
echo done
