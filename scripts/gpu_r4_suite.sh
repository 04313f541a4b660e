#!/bin/bash
# r4: the GPU suite + smoke on the current tree (after Python-only changes; the library is the
# final build, d5bbe5dc547e)
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-r4suite}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $OUT/pytest_gpu.log 2>&1; s=$?
tail -3 $OUT/pytest_gpu.log; [ $s -eq 0 ] || exit $s
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 11
tail -1 $OUT/smoke.log
