#!/bin/bash
# r5: the pair SLERP with non-temporal child stores (EDT_NT_SLERP_STORES, the in-tree build copied
# to build_variants/r5ntst.so) against the previous build (build_variants/default.so): one SLERP
# child (7B: stats, blend, far two-pass, lineage speculative), lerp / pair merge, the list step
# as a control; then the whole GPU suite on the new library.
set -o pipefail
O=gpurun_out/ntst
mkdir -p $O
for op in slerp stream; do
  echo "== $op" | tee -a $O/ab.log
  timeout -k 10 300 python3 -u scripts/kernel_variants.py --op $op --variants default,r5ntst --rounds 7 >> $O/ab.log 2>> $O/err.log \
      || { tail -20 $O/err.log; exit 1; }
done
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 \
    || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
