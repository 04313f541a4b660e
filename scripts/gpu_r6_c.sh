#!/bin/bash
# r6: the triangle layout folded into the needed-sums pass — the GPU suite on the new library,
# then the dense-graph probe against the previous library's separate Gram kernel.
set -o pipefail
O=gpurun_out/r6c
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 \
    || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 400 python3 -u scripts/triangle_probe.py > $O/triangle_probe.jsonl 2> $O/triangle_probe.err || { tail -20 $O/triangle_probe.err; exit 1; }
cat $O/triangle_probe.jsonl
echo done
