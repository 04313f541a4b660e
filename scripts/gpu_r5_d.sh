#!/bin/bash
# r5 step D: the whole GPU suite (sharded needed-sums path included).
set -o pipefail
O=gpurun_out/${R5_OUT:-r5l}
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 \
    || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
