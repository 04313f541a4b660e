#!/bin/bash
# r6: the new GPU tests (sharded dense graph on the triangle layout, two streams over one plan),
# then the multi-GPU line's code path at world 1 over RCCL, full size.
set -o pipefail
O=gpurun_out/r6f
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_virtual_ranks.py tests/test_gpu_shared_plan_threads.py > $O/pytest_new.log 2>&1 \
    || { tail -40 $O/pytest_new.log; exit 1; }
tail -1 $O/pytest_new.log
bash scripts/gpu_r6_e.sh
