#!/bin/bash
# GPU tests, the end-to-end (PCIe-inclusive) rates at 1.3B / 7B, and a rocprofv3 kernel trace of
# the sharded (RCCL, world 1) reduce schedule. Each GPU step under its own time limit, chained.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out; mkdir -p $OUT
R=$(pwd)
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; s=$?
tail -3 $OUT/pytest_gpu.log; [ $s -le 1 ] || exit $s
timeout -k 10 900 python -u scripts/e2e_large.py --what diloco,slerp --worker-dtype bf16 > $OUT/e2e_bf16.json 2> $OUT/e2e_bf16.err || exit $?
cat $OUT/e2e_bf16.json
timeout -k 10 600 python -u scripts/e2e_large.py --what diloco --worker-dtype f32 > $OUT/e2e_f32.json 2> $OUT/e2e_f32.err || exit $?
cat $OUT/e2e_f32.json
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $R/$OUT/prof_sharded -o sharded -- python3 $R/bench.py --gpus 1 --sharded --ops none --cpu-baseline-seconds 0 \
    --weak-companion 0 > $R/$OUT/prof_sharded.log 2>&1) || exit $?
grep '^{' $OUT/prof_sharded.log | cut -c1-400
find $OUT/prof_sharded -name "*kernel_stats*"
