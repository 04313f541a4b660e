#!/bin/bash
# r4: the ring Gram layout — population parity tests (every pair-graph shape vs per-child merges,
# configs[4] at its named shape), then the population probe under rocprofv3 (Gram pass time).
set -u
cd "$(dirname "$0")/.."
R=$(pwd); OUT=$R/gpurun_out/${TAG:-r4ring}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_config4.py tests/test_gpu_slerp_order.py \
    -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "population or config4 or order" \
    > $OUT/pytest_pop.log 2>&1; s=$?
tail -3 $OUT/pytest_pop.log; [ $s -eq 0 ] || exit $s
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $OUT/pop -o pop -- python3 $R/scripts/pop_slerp_probe.py --rounds 3 > $OUT/pop_probe.log 2>&1) || { tail -5 $OUT/pop_probe.log; exit 9; }
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $OUT/popring -o pop -- python3 $R/scripts/pop_slerp_probe.py --rounds 3 --pairs ring > $OUT/pop_probe_ring.log 2>&1) || { tail -5 $OUT/pop_probe_ring.log; exit 10; }
grep -v "^[EW]20" $OUT/pop_probe_ring.log | grep -v amdgpu | head -4
grep -v "^[EW]20" $OUT/pop_probe.log | grep -v amdgpu | head -4
python3 - $OUT/pop/pop_kernel_stats.csv $OUT/popring/pop_kernel_stats.csv <<'PY'
import csv, sys
for f in sys.argv[1:]:
    print(f)
    for r in csv.DictReader(open(f)):
        if "slerp" in r["Name"]:
            print(" ", r["Name"][:80], r["Calls"], round(float(r["AverageNs"]) / 1e6, 3))
PY
