#!/bin/bash
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r4popdt; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider -k "pair_graphs" > $OUT/pytest.log 2>&1; s=$?
tail -3 $OUT/pytest.log; exit $s
