# A/B of the split-halves addressing in the fused outer step, three dtype regimes, one process each
set -u
for cfg in "f32 f32" "f32 bf16" "bf16 bf16"; do
  set -- $cfg
  timeout -k 10 300 python scripts/kernel_variants.py --variants split0,split1,split1_nt0 --rounds 5 --tdt $1 --wdt $2 \
      > gpurun_out/split_$1_$2.json 2>/dev/null || exit 1
done
